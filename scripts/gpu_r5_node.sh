# round 5: bench.py's node section rehearsed on one GPU (2 ranks share cuda:0) + the 1-GPU headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_bench_gpu.py > gpurun_out/r5_node_test.log 2>&1 || { tail -40 gpurun_out/r5_node_test.log; exit 3; }
tail -3 gpurun_out/r5_node_test.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/r5_bench1.log 2>&1 || { tail -5 gpurun_out/r5_bench1.log; exit 4; }
grep '^{' gpurun_out/r5_bench1.log
