# round 4: TP tests after the tile sweep (fused exchange at 2/4/8 ranks on one GPU), then the probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py -k "allreduce or tensor_parallel or tp_group" -x -v --timeout 400 --timeout-method thread > gpurun_out/r4_tp_tests2.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r4_tp_tests2.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r4_tp_tests2.log
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_70b_v2.log 2>&1 || exit 2
grep -h '^{' gpurun_out/r4_tp_probe_70b_v2.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_8b_v2.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r4_tp_probe_8b_v2.log
