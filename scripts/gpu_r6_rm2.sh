# round 6: the single decode weight layout with its swept row-major tiles: bench A/B vs tiled, then config 5's eviction
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lay in single tiled single; do
  timeout -k 10 400 python -u bench.py --decode-weights $lay > gpurun_out/r6_rm_bench.log 2>&1 || { tail -20 gpurun_out/r6_rm_bench.log; exit 2; }
  grep '^{' gpurun_out/r6_rm_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); n=d['notes']; print(json.dumps({'layout': '$lay', 'req_s': d['value'], 'prefill_ms': round(n['rank0_prefill_s']/d['steps']*1e3,1), 'decode_ms': round(n['rank0_decode_s']/(d['steps']*127)*1e3,3)}))" | tee -a gpurun_out/r6_rm2_ab.jsonl
done
timeout -k 10 600 python -u bench/kv_eviction_bench.py --preset llama3-8b --requests 6000 --ttl 30 > gpurun_out/r6_evict2.log 2>&1 || { tail -5 gpurun_out/r6_evict2.log; exit 3; }
grep kv_eviction gpurun_out/r6_evict2.log
