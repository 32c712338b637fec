# round 6: in-graph decode-tile A/B on the headline bench (Llama-3-8B, 32 rows): each override is one bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {
  DIE_TILE_OVERRIDE="$1" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r6g.log 2>&1 || { tail -20 gpurun_out/r6g.log; exit 2; }
  grep '^{' gpurun_out/r6g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); n=d['notes']; print(json.dumps({'override': '$1', 'req_s': d['value'], 'decode_ms': round(n['rank0_decode_s']/(d['steps']*127)*1e3,4)}))" | tee -a gpurun_out/r6g_tiles.jsonl
}
run ""
for ov in "4096,14336,3,32=64,256,4" "4096,14336,3,32=128,128,8" "4096,14336,3,32=64,128,8" "4096,14336,3,32=32,256,2" \
          "4096,4096,3,32=32,128,2" "4096,4096,3,32=64,256,4" "4096,4096,3,32=32,256,4" \
          "6144,4096,2,32=48,128,2" "6144,4096,2,32=64,256,2" "6144,4096,2,32=48,256,4" ; do
  run "$ov"
done
run ""
for ov in "14336,4096,4,32=112,128,1" "4096,14336,3,32=128,64,8" "6144,4096,2,32=32,256,2" "4096,4096,3,32=64,128,2"; do
  run "$ov"
done
run ""
