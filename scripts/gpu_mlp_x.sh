set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "mlp_decode_persistent" -x -q --timeout 120 --timeout-method thread > gpurun_out/mlpx_test.log 2>&1 &&
DIE_MLP_XMODE=1 timeout -k 10 200 python bench/micro_mlp_decode.py 32 > gpurun_out/mlpx_1.jsonl 2>&1 &&
DIE_MLP_XMODE=2 timeout -k 10 200 python bench/micro_mlp_decode.py 32 > gpurun_out/mlpx_2.jsonl 2>&1 &&
DIE_MLP_XMODE=1 timeout -k 10 200 python bench/micro_mlp_decode.py 32 >> gpurun_out/mlpx_1.jsonl 2>&1 &&
DIE_MLP_XMODE=2 timeout -k 10 200 python bench/micro_mlp_decode.py 32 >> gpurun_out/mlpx_2.jsonl 2>&1
