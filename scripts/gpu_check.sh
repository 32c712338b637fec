set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gputests2.log 2>&1 ; echo "TESTS_EXIT $?" >> gpurun_out/gputests2.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke2.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --verbose > gpurun_out/bench2.log 2>&1
echo "BENCH_EXIT $?" >> gpurun_out/bench2.log
