set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench/micro_allreduce.py > gpurun_out/micro_allreduce.jsonl 2>gpurun_out/micro_allreduce.err &&
timeout -k 10 600 python bench/disagg_bench.py --steps 3 --warmup 1 > gpurun_out/disagg_bench.jsonl 2>gpurun_out/disagg_bench.err
