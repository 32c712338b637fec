set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/moe_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/moe_tests.log; exit 1; }
tail -1 gpurun_out/moe_tests.log
for v in 128 32; do
  DIE_MOE_DECODE_MAX_T=$v timeout -k 10 500 python bench.py --preset mixtral-8x7b --batch 64 --steps 1 --warmup 1 > gpurun_out/moe_b64_$v.log 2>&1 || exit 2
  echo "max_t=$v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|rank0_decode_s": [0-9.]*\|rank0_prefill_s": [0-9.]*' gpurun_out/moe_b64_$v.log | tr '\n' ' ')"
done
