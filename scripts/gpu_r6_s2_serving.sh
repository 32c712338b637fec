# final tree, serving paths: config 2 over RPC (client -> coordinator -> worker), config 3 as two worker processes
# (prefill -> decode through the IPC landing zone, one GPU), Poisson arrivals at 40 req/s
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench/serve_bench.py --mode llm --gpus 1 > gpurun_out/s2_serve_llm.log 2>&1 || { tail -10 gpurun_out/s2_serve_llm.log; exit 1; }
grep '^{' gpurun_out/s2_serve_llm.log | cut -c1-300
timeout -k 10 500 python bench/disagg_serve_bench.py --log-dir gpurun_out > gpurun_out/s2_disagg.jsonl 2> gpurun_out/s2_disagg.err || { echo "DISAGG FAILED"; tail -5 gpurun_out/s2_disagg.err; exit 2; }
cut -c1-300 gpurun_out/s2_disagg.jsonl
timeout -k 10 600 python -u bench/poisson_bench.py --rates 40 --modes auto --requests 300 > gpurun_out/s2_poisson.log 2>&1 || { tail -10 gpurun_out/s2_poisson.log; exit 3; }
grep '^{' gpurun_out/s2_poisson.log | cut -c1-300
