# timed-window kernel table of the Mixtral-8x7B bench (config 5's model, batch 32)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mxp -o mx -- python3 $R/bench.py --preset mixtral-8x7b --steps 1 --warmup 1 > gpurun_out/mxp.log 2>&1 || { tail -5 gpurun_out/mxp.log; exit 1; }
grep '^{' gpurun_out/mxp.log
python3 scripts/prof_window.py $(find gpurun_out/mxp -name '*kernel_trace.csv' | head -1) "bench.py Mixtral-8x7B timed wave" 20 --per 127 > gpurun_out/mxp_window.md
head -24 gpurun_out/mxp_window.md
rm -rf gpurun_out/mxp
