# batch-128 A/B on one box: queued decode windows on/off, XCD-aware prefill attention on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { echo -n "$1 "; shift; timeout -k 10 400 "$@" > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|rank0_decode_s": [0-9.]*\|rank0_prefill_s": [0-9.]*' gpurun_out/ab.log | tr '\n' ' '; echo; }
for rep in 1 2; do
run "b128 async xcd " python bench.py --batch 128 --steps 2 --warmup 1
run "b128 sync  xcd " python bench.py --batch 128 --steps 2 --warmup 1 --no-async-decode
DIE_PF_XCD=0 run "b128 async hw  " python bench.py --batch 128 --steps 2 --warmup 1
done
