# 16-row activation image A/B: kernel tests, micro (dense M=16/32, Mixtral grouped), Mixtral bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm_decode or moe" --timeout 120 --timeout-method thread > gpurun_out/xr16_tests.log 2>&1 || exit 1
for m in 8 16 32; do for x in 0 1; do
  DIE_GD_XR16=$x timeout -k 10 200 python -u bench/micro_gemm_decode.py $m moe >> gpurun_out/xr16_micro.jsonl 2>/dev/null || exit 2
done; done
DIE_GD_XR16=0 timeout -k 10 400 python bench.py --preset mixtral-8x7b --steps 1 --warmup 1 > gpurun_out/xr16_mixtral0.log 2>&1 || exit 3
DIE_GD_XR16=1 timeout -k 10 400 python bench.py --preset mixtral-8x7b --steps 1 --warmup 1 > gpurun_out/xr16_mixtral1.log 2>&1 || exit 4
