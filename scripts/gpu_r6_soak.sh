# round 6: serving soak through client -> coordinator -> worker (Llama-3-8B): 4,000 mixed requests (text and token ids,
# greedy and sampled, shared prefixes, a KV pool small enough to preempt and evict), text in the pre/post-processing pool;
# every request must return its token count and no KV block may stay held
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench/stress.py --preset llama3-8b --requests 4000 --concurrency 128 --kv-blocks 3000 --text-frac 0.3 --preproc-processes 4 > gpurun_out/r6_soak.log 2>&1 || { tail -20 gpurun_out/r6_soak.log; exit 1; }
grep '^{' gpurun_out/r6_soak.log
