# prefill attention: NW = 4 (two 4-wave workgroups per CU) vs 8 under the XCD-aware order, then the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for nw in 8 4 8 4; do
  for shp in "32 512" "4 4096" "1 8192"; do
    echo -n "nw=$nw " ; DIE_PF_NW=$nw timeout -k 10 120 python bench/micro_attn_prefill.py $shp || exit 2
  done
done
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/pfnw_bench.log 2>&1 || { tail -30 gpurun_out/pfnw_bench.log; exit 3; }
tail -1 gpurun_out/pfnw_bench.log
