set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_expert_parallel_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/xr16b_tests.log 2>&1 || exit 1
for m in 8 32; do
  timeout -k 10 200 python -u bench/micro_gemm_decode.py $m moe >> gpurun_out/xr16b_micro.jsonl 2>/dev/null || exit 2
done
