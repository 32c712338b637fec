# disaggregation on one GPU: IPC landing-zone serving tests, then the two-process bench (direct gather into the
# reserved slot, the default) and the staged path (DIE_KV_DIRECT=0) for A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_serving_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/disagg_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/disagg_tests.log | head -20; tail -30 gpurun_out/disagg_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/disagg_tests.log
timeout -k 10 500 python bench/disagg_serve_bench.py --log-dir gpurun_out > gpurun_out/disagg_serve.jsonl 2> gpurun_out/disagg_serve.err || { echo "DISAGG BENCH FAILED"; tail -5 gpurun_out/disagg_serve.err; exit 3; }
DIE_KV_DIRECT=0 timeout -k 10 500 python bench/disagg_serve_bench.py --log-dir gpurun_out >> gpurun_out/disagg_serve.jsonl 2>> gpurun_out/disagg_serve.err || { echo "DISAGG BENCH STAGED FAILED"; tail -5 gpurun_out/disagg_serve.err; exit 4; }
cat gpurun_out/disagg_serve.jsonl
