# the headline workload over the real RPC path (client -> coordinator -> GPU worker process)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python bench/serve_bench.py --mode llm --gpus 1 --concurrency 32 > gpurun_out/serve_llm.log 2>&1 || exit 1
