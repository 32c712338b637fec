# round 4 A/B: 70B TP=8 probe with valid (<= 128 statistics tiles) shard tiles, the 8B micro-sweep winners in the
# real graph (DIE_TILE_OVERRIDE) against the table, disaggregation with / without the IPC completion event
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/ab_tp70.log 2>&1 || exit 4
grep -h '^{' gpurun_out/ab_tp70.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ab_bench_base.log 2>&1 || { tail -5 gpurun_out/ab_bench_base.log; exit 3; }
grep '^{' gpurun_out/ab_bench_base.log
DIE_TILE_OVERRIDE="4096,4096,3,32=32,256,2;14336,4096,4,32=128,128,1;4096,14336,3,32=64,128,4" timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ab_bench_tiles.log 2>&1 || { tail -5 gpurun_out/ab_bench_tiles.log; exit 5; }
grep '^{' gpurun_out/ab_bench_tiles.log
DIE_TILE_OVERRIDE="14336,4096,4,32=128,128,1" timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ab_bench_gu.log 2>&1 || { tail -5 gpurun_out/ab_bench_gu.log; exit 6; }
grep '^{' gpurun_out/ab_bench_gu.log
DIE_TILE_OVERRIDE="4096,4096,3,32=32,256,2" timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ab_bench_o.log 2>&1 || { tail -5 gpurun_out/ab_bench_o.log; exit 7; }
grep '^{' gpurun_out/ab_bench_o.log
DIE_KV_IPC_EVENT=0 timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/ab_disagg_noevent.jsonl 2> gpurun_out/ab_disagg.err || { tail -5 gpurun_out/ab_disagg.err; exit 8; }
cat gpurun_out/ab_disagg_noevent.jsonl
timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/ab_disagg_event.jsonl 2>> gpurun_out/ab_disagg.err || { tail -5 gpurun_out/ab_disagg.err; exit 9; }
cat gpurun_out/ab_disagg_event.jsonl
