# round 5: uneven split-K (split counts that do not divide K's slots) — tests, 70B TP=8 qkv sweep, probe A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_decode or attn_decode_fused" > gpurun_out/us_tests.log 2>&1 || { tail -30 gpurun_out/us_tests.log; exit 1; }
tail -2 gpurun_out/us_tests.log
timeout -k 10 300 python bench/micro_tp_tiles.py --shapes 70b_tp8 --proj qkv --splits 2,3,4,5,6 > gpurun_out/us_sweep.jsonl 2>&1 || { tail -5 gpurun_out/us_sweep.jsonl; exit 2; }
grep best gpurun_out/us_sweep.jsonl
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench/tp_probe.py > gpurun_out/us_$name.log 2>&1 || { tail -5 gpurun_out/us_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/us_$name.log | tail -1 | grep -o '"decode_ms_per_step": [0-9.]*')"
}
run base_a X=1 && run sk5_a DIE_TILE_OVERRIDE="1280,8192,2,32=32,256,5" && run base_b X=1 && run sk5_b DIE_TILE_OVERRIDE="1280,8192,2,32=32,256,5"
