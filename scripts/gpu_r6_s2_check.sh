# session-2 sanity check of the rebuilt extensions: kernel tests, smoke, bench (N=1 defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s2_kernels.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/s2_kernels.log; exit 1; }
tail -2 gpurun_out/s2_kernels.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_smoke.log 2>&1 || { tail -5 gpurun_out/s2_smoke.log; exit 2; }
tail -1 gpurun_out/s2_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/s2_bench.log 2>&1 || { tail -5 gpurun_out/s2_bench.log; exit 3; }
grep '^{' gpurun_out/s2_bench.log | cut -c1-400
