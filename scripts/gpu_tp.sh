# tensor parallelism on the one GPU: IPC all-reduce / all-gather at 2/4/8 ranks, TP engines (2 ranks eager,
# 4 and 8 ranks with hipGraph decode) against TP=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py -k "allreduce or tensor_parallel" -x -v --timeout 400 --timeout-method thread > gpurun_out/tp_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tp_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/tp_tests.log
