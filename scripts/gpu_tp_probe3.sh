set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tp3_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/tp_probe_70b_v3.log 2>&1 || exit 2
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tpprof -o p -- python3 $GRAFT_REPO_ROOT/bench/tp_probe.py --preset llama3-70b --tp 8 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/tp_probe_prof.log 2>&1 || exit 3
