# session-2 final tree: the driver's round-end GPU steps (whole GPU suite in one process, smoke, bench), then the
# headline bench's timed-window kernel table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/s2f_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/s2f_tests.log | head -20; tail -30 gpurun_out/s2f_tests.log; exit 1; }
tail -2 gpurun_out/s2f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2f_smoke.log 2>&1 || { tail -5 gpurun_out/s2f_smoke.log; exit 2; }
tail -1 gpurun_out/s2f_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/s2f_bench.log 2>&1 || { tail -5 gpurun_out/s2f_bench.log; exit 3; }
grep '^{' gpurun_out/s2f_bench.log | cut -c1-300
export DIE_PROF_MARKERS=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p7b -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/p7b.log 2>&1 || { tail -5 gpurun_out/p7b.log; exit 4; }
python3 scripts/prof_window.py $(find /tmp/p7b -name '*kernel_trace.csv' | head -1) "bench.py timed region (2 waves), round 6 final tree (prefill residual add in the GEMM epilogue)" 30 --per 254 > gpurun_out/p7b_window.md
head -24 gpurun_out/p7b_window.md
