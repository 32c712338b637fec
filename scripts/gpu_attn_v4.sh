set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn" -x -v --timeout 120 --timeout-method thread > gpurun_out/v4_tests.log 2>&1
