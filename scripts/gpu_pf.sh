# prefill attention: numerics tests, then the micro bench at 32x512 / 4x4096 / 1x8192 for each DIE_ATTN_PF value in $PFS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
for v in ${PFS:-0 2}; do
  for shape in "32 512" "4 4096" "1 8192"; do
    DIE_ATTN_PF=$v timeout -k 10 120 python bench/micro_attn_prefill.py $shape > gpurun_out/pf_$v.log 2>&1 || { echo "BENCH FAILED pf=$v $shape"; tail -5 gpurun_out/pf_$v.log; exit 2; }
    echo "pf=$v $(cat gpurun_out/pf_$v.log)"
  done
done
