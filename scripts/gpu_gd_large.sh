# decode GEMM at M <= 128: kernel numerics, the 8B-shape oracle, then the large-M microbenchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_oracle_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gdl_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gdl_tests.log; exit 1; }
tail -1 gpurun_out/gdl_tests.log
timeout -k 10 600 python bench/micro_gemm_decode_large.py ${MS:-32 64 128} > gpurun_out/gdl_micro.jsonl 2> gpurun_out/gdl_micro.err || { echo "MICRO FAILED"; tail -5 gpurun_out/gdl_micro.err; exit 2; }
