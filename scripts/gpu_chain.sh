set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/micro_gemm_decode.py 32 chain > gpurun_out/chain.jsonl 2> gpurun_out/chain.err || exit 1
timeout -k 10 300 python -u bench/micro_gemm_decode.py 8 chain >> gpurun_out/chain.jsonl 2>> gpurun_out/chain.err || exit 2
