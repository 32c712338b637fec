# prefill GEMM table with the down projection's beta = 1 winners vs the round-5 table, interleaved on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['notes']['rank0_prefill_s'], d['notes']['rank0_decode_s'])"; }
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/tab_new_$i.log 2>&1 || { tail -5 gpurun_out/tab_new_$i.log; exit 1; }
  show gpurun_out/tab_new_$i.log new
  timeout -k 10 300 python scripts/bench_with_table.py bench/gemm_table_gfx950_round5.csv > gpurun_out/tab_old_$i.log 2>&1 || { tail -5 gpurun_out/tab_old_$i.log; exit 2; }
  show gpurun_out/tab_old_$i.log old
done
