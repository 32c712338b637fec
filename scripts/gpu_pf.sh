# prefill attention: numerics tests, then the micro bench at 32 x 512 / 4 x 4,096 / 1 x 8,192 for the
# 8-wave (default) and 4-wave (DIE_PF_NW=4) workgroup shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
for nw in 8 4; do
  for shape in "32 512" "4 4096" "1 8192"; do
    DIE_PF_NW=$nw timeout -k 10 120 python bench/micro_attn_prefill.py $shape > gpurun_out/pf.log 2>&1 || { echo "BENCH FAILED $shape"; tail -5 gpurun_out/pf.log; exit 2; }
    echo "nw=$nw $(grep '^{' gpurun_out/pf.log)"
  done
done
