# decode at M <= 128: kernel + oracle + engine GPU tests, then bench at batch 32 / 64 / 128
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_oracle_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/m128_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/m128_tests.log; exit 1; }
tail -1 gpurun_out/m128_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/m128_b32.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/m128_b64.log 2>&1 || exit 3
timeout -k 10 400 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/m128_b128.log 2>&1 || exit 4
for b in 32 64 128; do grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|rank0_decode_s": [0-9.]*\|rank0_prefill_s": [0-9.]*' gpurun_out/m128_b$b.log | tr '\n' ' '; echo; done
