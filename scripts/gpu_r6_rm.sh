# round 6: decode on the row-major weights (decode_weight_layout = single, config 5's capacity mode): 8B tile sweep
# for that layout, and the headline bench with single vs tiled on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/micro_tp_tiles.py --shapes 8b --row-major > gpurun_out/r6_8b_rm_tiles.jsonl 2>&1 || { tail -20 gpurun_out/r6_8b_rm_tiles.jsonl; exit 1; }
grep '"best"' gpurun_out/r6_8b_rm_tiles.jsonl
for lay in single tiled single; do
  timeout -k 10 400 python -u bench.py --decode-weights $lay > gpurun_out/r6_rm_bench.log 2>&1 || { tail -20 gpurun_out/r6_rm_bench.log; exit 2; }
  grep '^{' gpurun_out/r6_rm_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); n=d['notes']; print(json.dumps({'layout': '$lay', 'req_s': d['value'], 'prefill_ms': round(n['rank0_prefill_s']/d['steps']*1e3,1), 'decode_ms': round(n['rank0_decode_s']/(d['steps']*127)*1e3,3)}))" | tee -a gpurun_out/r6_rm_ab.jsonl
done
