set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench/micro_mixed_gemm.py > gpurun_out/micro_mixed_gemm.jsonl 2>gpurun_out/micro_mixed_gemm.err
