# config 5 on its own model: Mixtral-8x7B (93 GB of weights), KV pool in the HBM left; 800 distinct 2,048-token
# prefixes > the pool (~1.2 M tokens); prefix caching on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1100 python -u bench/kv_eviction_bench.py --preset mixtral-8x7b --prefixes 800 --requests 3000 --ttl 30 > gpurun_out/r4_evict_mixtral.log 2>&1 || { tail -5 gpurun_out/r4_evict_mixtral.log; exit 1; }
grep kv_eviction gpurun_out/r4_evict_mixtral.log
