# headline bench only (1 GPU), 5 timed waves
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_only.log 2>&1
