# round-end style check: all GPU tests, smoke, bench, the serving path through the coordinator, then a
# kernel-stats profile of one timed wave
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/fin_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/fin_tests.log; tail -5 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/fin_smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/fin_bench.log 2>&1 || exit 3
grep '^{' gpurun_out/fin_bench.log
timeout -k 10 600 python bench/serve_bench.py --mode llm --workers 1 --concurrency 32 --requests 96 > gpurun_out/fin_serve_llm.jsonl 2> gpurun_out/fin_serve_llm.err || { tail -5 gpurun_out/fin_serve_llm.err; exit 4; }
cat gpurun_out/fin_serve_llm.jsonl
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/finprof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/fin_prof.log 2>&1 || exit 5
