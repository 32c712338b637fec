set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_serving_gpu.py -x -v -s --timeout 280 --timeout-method thread > gpurun_out/serving_gpu.log 2>&1
