set -o pipefail
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench.log 2>&1
echo "EXIT $?" >> gpurun_out/prof_bench.log
