# headline bench: decode window (steps per queued hipGraph window) 8 (default) vs 16 vs 32, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['notes']['rank0_prefill_s'], d['notes']['rank0_decode_s'])"; }
for i in 1 2; do
  for w in 8 16 32; do
    timeout -k 10 300 python bench.py --decode-window $w > gpurun_out/win_${w}_$i.log 2>&1 || { tail -5 gpurun_out/win_${w}_$i.log; exit 1; }
    show gpurun_out/win_${w}_$i.log "window$w"
  done
done
