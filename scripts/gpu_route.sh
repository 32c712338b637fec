# MoE decode changes: kernel + engine tests, then the Mixtral and 8B benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_expert_parallel_gpu.py -x -v -k "moe or mixtral or engine or tensor_parallel or expert" --timeout 200 --timeout-method thread > gpurun_out/route_tests.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/route_mixtral.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/route_8b.log 2>&1 || exit 3
