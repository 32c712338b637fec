# persistent decode step vs five launches per layer at 1 / 4 / 8 / 16 / 32 decode rows (Llama-3-8B, 32 layers)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in 1 4 8 16 32; do
  timeout -k 10 200 python -u bench/micro_decode_persistent.py 32 20 $m > gpurun_out/dp_rows_$m.log 2>&1 || { tail -5 gpurun_out/dp_rows_$m.log; exit 1; }
  grep '^{' gpurun_out/dp_rows_$m.log | sed "s/^/rows=$m /"
done
