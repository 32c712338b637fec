# round 6: config 5 eviction at full HBM with the decode weights in one layout (auto under kv_capacity_priority) vs the
# tile-order copies; prefill GEMM clock (PMC GRBM_GUI_ACTIVE over each dispatch: is 1.5 PF/s a clock ceiling?)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/kv_eviction_bench.py --preset llama3-8b --requests 6000 --ttl 30 > gpurun_out/r6d_evict_auto.log 2>&1 || { tail -5 gpurun_out/r6d_evict_auto.log; exit 1; }
grep kv_eviction gpurun_out/r6d_evict_auto.log
timeout -k 10 600 python -u bench/kv_eviction_bench.py --preset llama3-8b --requests 6000 --ttl 30 --decode-weights tiled > gpurun_out/r6d_evict_tiled.log 2>&1 || { tail -5 gpurun_out/r6d_evict_tiled.log; exit 2; }
grep kv_eviction gpurun_out/r6d_evict_tiled.log
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmcclk -o clk -- python3 $R/bench/micro_prefill_gemm.py > gpurun_out/r6d_pmc_clk.log 2>&1 || { tail -5 gpurun_out/r6d_pmc_clk.log; exit 3; }
grep '^{' gpurun_out/r6d_pmc_clk.log
find gpurun_out/pmcclk -name '*counter_collection.csv' -exec cp {} gpurun_out/r6d_pmc_clk.csv \;
head -3 gpurun_out/r6d_pmc_clk.csv
rm -rf gpurun_out/pmcclk
