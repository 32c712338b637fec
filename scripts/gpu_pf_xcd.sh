# prefill attention: numerics tests, then A/B of the XCD-aware workgroup order (DIE_PF_XCD=0/1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "prefill or attention" --timeout 120 --timeout-method thread > gpurun_out/pfx_tests.log 2>&1 || { tail -30 gpurun_out/pfx_tests.log; exit 1; }
tail -2 gpurun_out/pfx_tests.log
for x in 0 1 0 1; do
  for shp in "32 512" "8 2048" "4 4096" "1 8192"; do
    echo -n "xcd=$x " ; DIE_PF_XCD=$x timeout -k 10 120 python bench/micro_attn_prefill.py $shp || exit 2
  done
done
