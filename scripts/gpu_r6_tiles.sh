# round 6: in-graph tile A/B of the 70B TP=8 shard's decode GEMMs (DIE_TILE_OVERRIDE; mode 6 = split-K SiLU gate/up)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for ov in "" "8192,3584,3,32=64,128,2" "8192,3584,3,32=128,128,4" "3584,8192,6,32=112,128,4" "3584,8192,6,32=128,128,4" "8192,1024,3,32=64,128,2" "8192,3584,3,32=64,256,2" "1280,8192,2,32=32,256,5" ""; do
  DIE_TILE_OVERRIDE="$ov" timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 3 --warmup 1 > gpurun_out/r6t.log 2>&1 || { tail -20 gpurun_out/r6t.log; exit 3; }
  grep -h '^{' gpurun_out/r6t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['tile_override']='$ov'; print(json.dumps(d))" | tee -a gpurun_out/r6t_tiles.jsonl | cut -c1-120
  grep -h '^{' gpurun_out/r6t.log | grep -o '"decode_ms_per_step": [0-9.]*\|"down_tile": \[[0-9, ]*\]\|"o_tile": \[[0-9, ]*\]'
done
