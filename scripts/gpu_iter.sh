# development loop: kernel + engine GPU tests, optional micro benches ($MICRO), then the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/it_tests.log; exit 1; }
tail -1 gpurun_out/it_tests.log
for m in $MICRO; do
  timeout -k 10 200 python bench/$m.py > gpurun_out/it_$m.log 2>&1 || { echo "MICRO $m FAILED"; tail -5 gpurun_out/it_$m.log; exit 2; }
  grep '^{' gpurun_out/it_$m.log
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/it_bench.log 2>&1 || exit 3
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|rank0_decode_s": [0-9.]*\|rank0_prefill_s": [0-9.]*' gpurun_out/it_bench.log
