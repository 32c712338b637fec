# round 4 first check on a fresh box: full GPU suite (release build), the persistent step's tests on the
# diagnostics build, the driver bench, and the two-process disaggregation bench (uncached landing zone)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/r4_tests.log; tail -5 gpurun_out/r4_tests.log; exit 1; }
tail -1 gpurun_out/r4_tests.log
DIE_C_DIAG=1 timeout -k 10 300 python -u -m pytest tests/test_decode_persistent_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_persistent_diag.log 2>&1 || { tail -5 gpurun_out/r4_persistent_diag.log; exit 2; }
tail -1 gpurun_out/r4_persistent_diag.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r4_bench.log 2>&1 || { tail -5 gpurun_out/r4_bench.log; exit 3; }
grep '^{' gpurun_out/r4_bench.log
timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/r4_disagg.jsonl 2> gpurun_out/r4_disagg.err || { tail -5 gpurun_out/r4_disagg.err; exit 4; }
cat gpurun_out/r4_disagg.jsonl
DIE_KV_ZONE_UNCACHED=0 timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/r4_disagg_cached.jsonl 2>> gpurun_out/r4_disagg.err || { tail -5 gpurun_out/r4_disagg.err; exit 5; }
cat gpurun_out/r4_disagg_cached.jsonl
