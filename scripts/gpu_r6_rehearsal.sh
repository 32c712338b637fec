# exactly the driver's round-end GPU steps: the whole GPU suite in one process, smoke, bench (N=1 defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6r_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/r6r_tests.log | head -20; tail -30 gpurun_out/r6r_tests.log; exit 1; }
tail -2 gpurun_out/r6r_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6r_smoke.log 2>&1 || { tail -5 gpurun_out/r6r_smoke.log; exit 2; }
tail -2 gpurun_out/r6r_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6r_bench.log 2>&1 || { tail -5 gpurun_out/r6r_bench.log; exit 3; }
grep '^{' gpurun_out/r6r_bench.log | cut -c1-300
