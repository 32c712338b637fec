#!/bin/bash
# GPU idle time inside the headline bench's timed region (2 waves): rocprofv3 kernel trace (kept in /tmp),
# summaries by scripts/prof_gaps.py and scripts/prof_window.py into gpurun_out/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/pg -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/pg.log 2>&1 || { tail -5 gpurun_out/pg.log; exit 1; }
T=$(find /tmp/pg -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_gaps.py $T --min-us 5 --top 15 > gpurun_out/pg_gaps.md
python3 scripts/prof_window.py $T "bench.py timed region (2 waves)" 30 --per 254 > gpurun_out/pg_window.md
cat gpurun_out/pg_gaps.md
