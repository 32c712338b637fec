# engine-level change check: engine / oracle / serving GPU tests, then the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_oracle_gpu.py tests/test_serving_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/it_tests.log; exit 1; }
tail -3 gpurun_out/it_tests.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/it_bench.log 2>&1 || { tail -30 gpurun_out/it_bench.log; exit 3; }
tail -1 gpurun_out/it_bench.log
