# HBM bytes per kernel in the bench's timed region: FETCH_SIZE and WRITE_SIZE in two passes (one TCC counter group
# each), with the kernel trace of the same run for the per-dispatch time (scripts/pmc_window.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pm_$C -o b -- python3 $R/bench.py --steps 1 --warmup 1 > gpurun_out/pm_$C.log 2>&1 || { tail -5 gpurun_out/pm_$C.log; exit 1; }
  python3 scripts/pmc_window.py $(find gpurun_out/pm_$C -name '*counter_collection.csv' | head -1) $(find gpurun_out/pm_$C -name '*kernel_trace.csv' | head -1) "bench.py timed wave, $C" --per 127 > gpurun_out/pm_$C.md
  head -14 gpurun_out/pm_$C.md
  rm -rf gpurun_out/pm_$C
done
