# round 6: the driver's N=4 run shape rehearsed with 4 ranks on one GPU (models scaled to fit one GPU's HBM: config 5
# and the TP wave on Llama-3-8B instead of Mixtral / 70B): 2 disaggregated pairs, 4 balanced workers, an 8B TP=4 wave
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u bench.py --gpus 4 --same-device --steps 2 --warmup 1 --cross-gpu-budget-s 900 --lb-preset llama3-8b --tp-wave-min-world 4 --tp-wave-preset llama3-8b --verbose > gpurun_out/r6n4_bench.log 2>&1 || { echo "EXIT $?"; tail -30 gpurun_out/r6n4_bench.log; exit 3; }
grep '^{' gpurun_out/r6n4_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['notes'].get('cross_gpu',{}); print(d['value'], d.get('cross_gpu_status')); print(json.dumps({k: (c.get(k) if k!='lb_serving' else {kk: c[k].get(kk) for kk in ('req_s','p50_latency_ms','p99_latency_ms','prefix_hit_rate','lru_evictions','dispatched_per_worker','error')}) for k in ('status','disagg','tp_wave','lb_serving') if k in c})[:4000])"
