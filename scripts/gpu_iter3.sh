set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/it3_kern.log 2>&1 || { echo "KERNEL TESTS FAILED" >> gpurun_out/it3_kern.log; exit 1; }
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/it3_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/it3_tests.log; exit 1; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/it3_bench.log 2>&1 || exit 2
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/it3_prof.log 2>&1 || exit 3
