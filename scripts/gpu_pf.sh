# prefill attention: numerics, then the micro at the bench shape and long prompts with an A/B knob ($KNOB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill or attn" -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
for v in 0 1; do for shp in "32 512" "4 4096" "1 8192"; do
  env ${KNOB:-X}=$v timeout -k 10 120 python bench/micro_attn_prefill.py $shp | sed "s/^/${KNOB:-X}=$v /" || exit 2
done; done
