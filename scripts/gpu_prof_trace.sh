# kernel trace of one timed bench wave (csv) for scripts/prof_gaps.py + stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/trace_bench.log 2>&1
