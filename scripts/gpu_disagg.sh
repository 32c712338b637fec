# disaggregation: serving GPU tests (IPC landing zone lifecycle + injected sender failure), IPC copy
# method micro (shader vs DMA), two-process prefill->decode bench with each copy method
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_serving_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dg_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/dg_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/dg_tests.log
timeout -k 10 300 python bench/micro_ipc_copy.py > gpurun_out/ipc_copy.jsonl 2> gpurun_out/ipc_copy.err || { echo "IPC MICRO FAILED"; tail -5 gpurun_out/ipc_copy.err; exit 2; }
cat gpurun_out/ipc_copy.jsonl
timeout -k 10 500 python bench/disagg_serve_bench.py --log-dir gpurun_out > gpurun_out/disagg_serve.jsonl 2> gpurun_out/disagg_serve.err || { echo "DISAGG BENCH FAILED"; tail -5 gpurun_out/disagg_serve.err; exit 3; }
DIE_KV_COPY=dma timeout -k 10 500 python bench/disagg_serve_bench.py --log-dir gpurun_out >> gpurun_out/disagg_serve.jsonl 2>> gpurun_out/disagg_serve.err || { echo "DISAGG BENCH DMA FAILED"; tail -5 gpurun_out/disagg_serve.err; exit 4; }
cat gpurun_out/disagg_serve.jsonl
