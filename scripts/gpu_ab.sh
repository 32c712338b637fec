# A/B of an env knob on the headline bench: tests first, then bench with $KNOB=0 and =1 (twice each, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_oracle_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/ab_tests.log
for rep in 1 2; do for v in 0 1; do
  env $KNOB=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/ab_$v.log 2>&1 || exit 2
  echo "$KNOB=$v $(grep -o '"value": [0-9.]*\|rank0_decode_s": [0-9.]*\|rank0_prefill_s": [0-9.]*' gpurun_out/ab_$v.log | tr '\n' ' ')"
done; done
