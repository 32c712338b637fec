# one-shot IPC all-reduce GPU tests (2 / 4 / 8 ranks sharing the GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/car_tests.log 2>&1
