# development loop: kernel + engine GPU tests, then the headline bench (A/B via env)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/it_tests.log; exit 1; }
tail -2 gpurun_out/it_tests.log
DIE_GD_TILED=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/it_bench_rowmajor.log 2>&1 || exit 3
DIE_GD_TILED=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/it_bench_tiled.log 2>&1 || exit 4
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|rank0_decode_s": [0-9.]*' gpurun_out/it_bench_rowmajor.log gpurun_out/it_bench_tiled.log
