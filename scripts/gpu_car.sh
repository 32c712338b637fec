set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py -k "allreduce or tensor_parallel" -x -v -s --timeout 280 --timeout-method thread > gpurun_out/car_test.log 2>&1
