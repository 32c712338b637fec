set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== 2-False then 8"; timeout -k 5 80 python -u -m pytest tests/test_engine_gpu.py -k "tensor_parallel and (llama-mini-tp-False-2-False or 8-True)" -x -v -s --timeout 70 --timeout-method thread > gpurun_out/dbg3_g.log 2>&1; echo "exit $?"; grep -E "\[tp 8\]|PASSED|FAILED|passed|failed" gpurun_out/dbg3_g.log | head -30
