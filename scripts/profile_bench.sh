#!/bin/bash
# rocprofv3 kernel trace + per-kernel stats of the bench (ARGS overrides the bench arguments, e.g.
# ARGS="--model mixtral-8x7b --steps 1 --warmup 1"). Output: gpurun_out/prof/, log gpurun_out/prof_bench.log
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS=${ARGS:-"--steps 1 --warmup 1"}
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py $ARGS > gpurun_out/prof_bench.log 2>&1
echo "EXIT $?" >> gpurun_out/prof_bench.log
