set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
AMD_LOG_LEVEL=1 timeout -k 10 400 python -u -m pytest tests/test_serving_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/dbg_serving.log 2>&1 || { echo "SERVING FAILED $?" >> gpurun_out/dbg_serving.log; exit 1; }
