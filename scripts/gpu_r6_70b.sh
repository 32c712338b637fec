# round 6: Llama-3-70B on ONE GPU (TP=1, decode on the row-major weights): tile sweep + the bench at its current tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/micro_tp_tiles.py --shapes 70b --row-major > gpurun_out/r6_70b_tiles.jsonl 2>&1 || { tail -20 gpurun_out/r6_70b_tiles.jsonl; exit 1; }
grep '"best"' gpurun_out/r6_70b_tiles.jsonl
timeout -k 10 500 python -u bench.py --preset llama3-70b --steps 2 --warmup 1 > gpurun_out/r6_70b_bench.log 2>&1 || { tail -20 gpurun_out/r6_70b_bench.log; exit 2; }
grep '^{' gpurun_out/r6_70b_bench.log | cut -c1-250
