set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profmx -o run -- python3 $R/bench.py --steps 1 --warmup 1 --preset mixtral-8x7b > $R/gpurun_out/profmx.log 2>&1
