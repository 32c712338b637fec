# round 5: driver-identical GPU steps (whole GPU suite in one process, smoke, bench N=1 defaults), then a
# kernel-stats profile of a short bench run (copied to profiles/ by hand)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/r5g_tests.log | head -20; tail -30 gpurun_out/r5g_tests.log; exit 1; }
tail -2 gpurun_out/r5g_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g_smoke.log 2>&1 || { tail -5 gpurun_out/r5g_smoke.log; exit 2; }
tail -2 gpurun_out/r5g_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5g_bench.log 2>&1 || { tail -5 gpurun_out/r5g_bench.log; exit 3; }
grep '^{' gpurun_out/r5g_bench.log | cut -c1-600
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r5g -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r5g_prof.log 2>&1 || { tail -5 gpurun_out/r5g_prof.log; exit 4; }
python scripts/prof_summary.py $(find /tmp/prof_r5g -name '*kernel_stats.csv' | head -1) "bench --steps 2 --warmup 1, round 5 tree" 24 > gpurun_out/r5g_kernel_stats.md
head -30 gpurun_out/r5g_kernel_stats.md
