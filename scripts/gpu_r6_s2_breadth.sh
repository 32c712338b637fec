# session-2 final tree (prefill residual add in the GEMM epilogue): breadth rows — batch 64 / 128, 8K prompts,
# Mixtral-8x7B, Llama-3-70B TP=1 — with the A/B of the new path on the 8K-prompt row (the most prefill-bound)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
line() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); n=d.get('notes',{}); print(json.dumps({'run': '$2', 'req_s': d.get('value'), 'p50_ms': d.get('p50_latency_ms'), 'prefill_ms_wave': round(n['rank0_prefill_s']/d['steps']*1e3,1), 'decode_ms_step': round(n['rank0_decode_s']/(d['steps']*(d['config']['gen_len']-1))*1e3,3), 'metric': d['metric'], 'config': d['config']}))" | tee -a gpurun_out/s2_breadth.jsonl | cut -c1-200; }
timeout -k 10 400 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/bs2_b64.log 2>&1 || exit 1; line gpurun_out/bs2_b64.log batch64
timeout -k 10 400 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/bs2_b128.log 2>&1 || exit 2; line gpurun_out/bs2_b128.log batch128
timeout -k 10 500 python bench.py --prompt-len 8192 --max-model-len 8448 --steps 2 --warmup 1 > gpurun_out/bs2_p8k.log 2>&1 || exit 3; line gpurun_out/bs2_p8k.log prompt8k
timeout -k 10 500 python bench.py --prompt-len 8192 --max-model-len 8448 --steps 2 --warmup 1 --no-gemm-residual > gpurun_out/bs2_p8k_off.log 2>&1 || exit 3; line gpurun_out/bs2_p8k_off.log prompt8k_no_gemm_residual
timeout -k 10 500 python bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/bs2_mixtral.log 2>&1 || exit 4; line gpurun_out/bs2_mixtral.log mixtral
timeout -k 10 500 python bench.py --preset llama3-70b --steps 2 --warmup 1 > gpurun_out/bs2_70b.log 2>&1 || exit 5; line gpurun_out/bs2_70b.log 70b_tp1
