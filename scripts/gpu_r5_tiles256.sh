# round 5: 256 norm-statistics tiles (wr = 32 residual projections at 8,192 columns): kernel tests, 70B TP=8
# o / down tile sweep, and the probe with the table's tiles vs wr = 32 tiles (DIE_TILE_OVERRIDE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rownorm or attn_decode_fused or tiled_weights or slab_residual" > gpurun_out/r5t_tests.log 2>&1 || { tail -30 gpurun_out/r5t_tests.log; exit 1; }
tail -2 gpurun_out/r5t_tests.log
timeout -k 10 300 python bench/micro_tp_tiles.py --shapes 70b_tp8 --proj o,down > gpurun_out/r5t_tiles.jsonl 2>/dev/null || exit 2
grep best gpurun_out/r5t_tiles.jsonl
grep '"tile": \[32' gpurun_out/r5t_tiles.jsonl | head -20
timeout -k 10 400 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r5t_probe_base.log 2>&1 || { tail -5 gpurun_out/r5t_probe_base.log; exit 3; }
grep '^{' gpurun_out/r5t_probe_base.log
DIE_TILE_OVERRIDE="8192,1024,3,32=32,256,1;8192,3584,3,32=32,128,1" timeout -k 10 400 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r5t_probe_wr32.log 2>&1 || { tail -5 gpurun_out/r5t_probe_wr32.log; exit 4; }
grep '^{' gpurun_out/r5t_probe_wr32.log
