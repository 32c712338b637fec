# round 6: the driver's N=2 run shape rehearsed on one GPU (2 ranks share cuda:0): Llama-3-8B timed region, then the
# node section at its default models — 8B disaggregation with the transport A/B, config 5 with Mixtral-8x7B workers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 2 --same-device --steps 2 --warmup 1 --cross-gpu-budget-s 800 --verbose > gpurun_out/r6n_bench2.log 2>&1 || { echo "EXIT $?"; tail -30 gpurun_out/r6n_bench2.log; exit 3; }
grep '^{' gpurun_out/r6n_bench2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['notes'].get('cross_gpu',{}); print(d['value'], d.get('cross_gpu_status')); print(json.dumps({k: c.get(k) for k in ('status','disagg','lb_serving')})[:3000])"
