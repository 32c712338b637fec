# round 6: TP decode windows + the occupancy-based residency rule (half-LDS ring) — kernel tests, IPC collectives,
# TP engine tests (2/4/8 ranks on one GPU, token-exact vs TP=1, windows mirrored, group fails as a unit), probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "half_ring or refuses or lm_head_argmax" -x -v --timeout 120 --timeout-method thread > gpurun_out/r6_tp_kern.log 2>&1 || { echo "KERNEL TESTS FAILED"; tail -40 gpurun_out/r6_tp_kern.log; exit 1; }
grep -cE "PASSED" gpurun_out/r6_tp_kern.log
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py -k "custom_allreduce or tensor_parallel or tp_group" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_tp_tests.log 2>&1 || { echo "TP TESTS FAILED"; tail -40 gpurun_out/r6_tp_tests.log; exit 2; }
grep -E "PASSED|FAILED" gpurun_out/r6_tp_tests.log
timeout -k 10 400 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r6_tp70.log 2>&1 || { tail -20 gpurun_out/r6_tp70.log; exit 3; }
grep -h '^{' gpurun_out/r6_tp70.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r6_tp8.log 2>&1 || { tail -20 gpurun_out/r6_tp8.log; exit 4; }
grep -h '^{' gpurun_out/r6_tp8.log
