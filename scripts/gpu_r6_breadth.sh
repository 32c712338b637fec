# round 6 final tree: breadth rows (batch 64 / 128, 8K prompts, Mixtral-8x7B, Llama-3-70B TP=1), the 70B TP=8 probe at
# batch 64 / 128 and with 16-step windows, the 70B TP=1 runner-up tiles in the graph
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
line() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); n=d.get('notes',{}); print(json.dumps({'run': '$2', 'req_s': d.get('value'), 'p50_ms': d.get('p50_latency_ms'), 'prefill_ms_wave': round(n['rank0_prefill_s']/d['steps']*1e3,1), 'decode_ms_step': round(n['rank0_decode_s']/(d['steps']*(d['config']['gen_len']-1))*1e3,3), 'metric': d['metric'], 'config': d['config']}))" | tee -a gpurun_out/r6_breadth.jsonl | cut -c1-200; }
timeout -k 10 400 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/br6_b64.log 2>&1 || exit 1; line gpurun_out/br6_b64.log batch64
timeout -k 10 400 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/br6_b128.log 2>&1 || exit 2; line gpurun_out/br6_b128.log batch128
timeout -k 10 500 python bench.py --prompt-len 8192 --max-model-len 8448 --steps 1 --warmup 1 > gpurun_out/br6_p8k.log 2>&1 || exit 3; line gpurun_out/br6_p8k.log prompt8k
timeout -k 10 500 python bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/br6_mixtral.log 2>&1 || exit 4; line gpurun_out/br6_mixtral.log mixtral
for b in 64 128; do
  timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --batch $b --steps 2 --warmup 1 > gpurun_out/br6_tp.log 2>&1 || exit 5
  grep -h '^{' gpurun_out/br6_tp.log | tee -a gpurun_out/r6_breadth_tp.jsonl | cut -c1-200
done
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 3 --warmup 1 --decode-window 16 > gpurun_out/br6_tp.log 2>&1 || exit 6
grep -h '^{' gpurun_out/br6_tp.log | tee -a gpurun_out/r6_breadth_tp.jsonl | cut -c1-200
for ov in "" "10240,8192,2,32=128,128,2" "28672,8192,4,32=128,128,1" "8192,28672,3,32=64,128,4"; do
  DIE_TILE_OVERRIDE="$ov" timeout -k 10 500 python bench.py --preset llama3-70b --steps 2 --warmup 1 > gpurun_out/br6_70b.log 2>&1 || exit 7; line gpurun_out/br6_70b.log "70b_tp1 $ov"
done
