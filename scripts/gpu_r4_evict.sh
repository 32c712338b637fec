# config 5's LRU KV eviction at full HBM (bench/kv_eviction_bench.py): Llama-3-8B, the KV pool takes the HBM left
# after the weights; 1,200 distinct 2,048-token prefixes (Zipf 0.6) > the pool; prefix caching on, then off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench/kv_eviction_bench.py --preset llama3-8b --requests 6000 --ttl 30 > gpurun_out/r4_evict_8b.log 2>&1 || { tail -5 gpurun_out/r4_evict_8b.log; exit 1; }
grep kv_eviction gpurun_out/r4_evict_8b.log
timeout -k 10 900 python -u bench/kv_eviction_bench.py --preset llama3-8b --requests 6000 --ttl 30 --no-prefix-cache > gpurun_out/r4_evict_8b_off.log 2>&1 || { tail -5 gpurun_out/r4_evict_8b_off.log; exit 2; }
grep kv_eviction gpurun_out/r4_evict_8b_off.log
