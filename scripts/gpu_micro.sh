set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench/micro_gemm_decode.py 32 > gpurun_out/micro_gd32.log 2>&1 || exit 2
