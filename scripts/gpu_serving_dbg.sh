set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DIE_DEBUG_IPC=1 timeout -k 10 170 python -u -m pytest tests/test_serving_gpu.py -x -v -s -k ipc --timeout 280 --timeout-method thread > gpurun_out/dbg_serving.log 2>&1
