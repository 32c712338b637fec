"""Config 5's KV-cache promise at full HBM: "LRU KV eviction at 288 GB" (the reference's
LRU/TTL cache is `/root/reference/src/kvstore.py:82-102,200-204`, its promise `/root/reference/README.md:14`).

One engine whose paged KV pool takes the HBM left after the weights (gpu_memory_fraction of the 288 GB, as a
serving worker sizes it), driven closed-loop by a shared-prefix workload whose DISTINCT prefixes hold more tokens
than the pool: P prefixes of L tokens ("system prompts"), each request = one prefix drawn from a Zipf
distribution + a unique suffix of S tokens, G generated tokens. Prefix blocks of finished requests stay cached
(ref-count 0, hashed) until the allocator needs their space; the least recently released go first (LRU), and
blocks released more than --ttl seconds ago are swept (TTL). Reported: pool GiB / blocks / tokens, the workload's
working set, req/s, prompt tokens/s, TTFT p50 / p99, prefix-hit tokens and hit rate, LRU evictions, TTL
evictions. --no-prefix-cache runs the same workload with caching off (every prompt prefilled in full).

    python bench/kv_eviction_bench.py [--preset llama3-8b] [--prefixes 1200] [--prefix-len 2048] [--requests 6000]
    python bench/kv_eviction_bench.py --dry-run ...   # host-only: the block manager's LRU over the same stream
"""

import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def workload(a):
    rng = random.Random(a.seed)
    vocab = 30000
    prefixes = [[rng.randrange(3, vocab) for _ in range(a.prefix_len)] for _ in range(a.prefixes)]
    w = [1.0 / (i + 1) ** a.zipf for i in range(a.prefixes)]
    picks = rng.choices(range(a.prefixes), weights=w, k=a.requests)
    reqs = [prefixes[p] + [rng.randrange(3, vocab) for _ in range(a.suffix_len)] for p in picks]
    return reqs, len(set(picks))


def dry_run(a, reqs, pool_blocks):
    """The native block manager alone over the request stream, one request at a time (no model)."""
    from src.engine.block_manager import KVBlockManager
    from src.engine.sequence import Sequence
    from src.preproc import SamplingParams

    bm = KVBlockManager(pool_blocks, 16, not a.no_prefix_cache)
    hit = tot = 0
    for i, r in enumerate(reqs):
        s = Sequence(f"r{i}", r, SamplingParams(max_tokens=a.gen_len))
        bm.allocate(s)
        hit += s.num_prefix_hit
        tot += len(r)
        s.num_computed = len(r)
        bm.register_prompt_blocks(s)
        bm.free(s)
    return {"hit_rate": round(hit / tot, 4), "kv": bm.stats()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--prefixes", type=int, default=1200)
    ap.add_argument("--prefix-len", type=int, default=2048)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--gen-len", type=int, default=16)
    ap.add_argument("--requests", type=int, default=6000)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--zipf", type=float, default=0.6)
    ap.add_argument("--ttl", type=float, default=60.0, help="seconds a released cached block may stay (0: none)")
    ap.add_argument("--gpu-memory-fraction", type=float, default=0.9)
    ap.add_argument("--max-batched-tokens", type=int, default=16384)
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--decode-weights", default="auto", choices=("auto", "tiled", "single"),
                    help="EngineConfig.decode_weight_layout; config 5 is KV-capacity bound, so auto = single")
    ap.add_argument("--dry-run", type=int, default=0, metavar="POOL_BLOCKS",
                    help="host-only LRU simulation over a pool of this many blocks")
    a = ap.parse_args()
    reqs, distinct = workload(a)
    if a.dry_run:
        print(json.dumps({"dry_run": True, "distinct_prefixes": distinct, **dry_run(a, reqs, a.dry_run)}))
        return

    import torch

    from src.config import EngineConfig
    from src.engine import LLMEngine
    from src.preproc import SamplingParams

    cfg = EngineConfig(max_num_seqs=a.concurrency, max_num_batched_tokens=a.max_batched_tokens, max_latency_ms=0.0,
                       enable_prefix_caching=not a.no_prefix_cache, kv_block_ttl_s=a.ttl or None,
                       gpu_memory_fraction=a.gpu_memory_fraction, kv_capacity_priority=True,
                       decode_weight_layout=a.decode_weights)
    t0 = time.perf_counter()
    eng = LLMEngine.from_preset(a.preset, device="cuda:0", cfg=cfg, max_model_len=a.prefix_len + a.suffix_len +
                                a.gen_len + 16)
    eng.eos_token_id = None
    init_s = time.perf_counter() - t0
    pool_tokens = eng.blocks.num_blocks * cfg.block_size
    sp = SamplingParams(max_tokens=a.gen_len, ignore_eos=True)
    ttft, done = [], [0]
    nxt = [0]

    def submit():
        i = nxt[0]
        nxt[0] += 1

        def fin(s):
            done[0] += 1
            ttft.append(s.ttft_ms())
            assert len(s.output_ids) == a.gen_len, (i, len(s.output_ids))
        eng.add_request(f"r{i}", reqs[i], sp, on_finish=fin)

    # warm-up outside the clock: a few requests with their own prefixes (graphs, hipBLASLt heuristics)
    rng = random.Random(99)
    eng.generate([[rng.randrange(3, 30000) for _ in range(a.prefix_len + a.suffix_len)] for _ in range(4)], sp)
    kv0 = eng.get_stats()["kv"]
    hits0, prompt0 = eng.stats["prefix_hit_tokens"], eng.stats["prompt_tokens"]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last_print = t0
    while nxt[0] < min(a.concurrency, len(reqs)):
        submit()
    while eng.has_work():
        before = done[0]
        eng.step()
        for _ in range(done[0] - before):
            if nxt[0] < len(reqs):
                submit()
        now = time.perf_counter()
        if now - last_print > 30:  # progress for long runs
            print(json.dumps({"progress": done[0], "elapsed_s": round(now - t0, 1)}), flush=True)
            last_print = now
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kv = eng.get_stats()["kv"]
    hit = eng.stats["prefix_hit_tokens"] - hits0
    prompt = eng.stats["prompt_tokens"] - prompt0
    ttft.sort()
    print(json.dumps({
        "bench": "kv_eviction_full_hbm", "preset": a.preset, "prefix_caching": not a.no_prefix_cache,
        "pool_gib": round(eng.pool.nbytes / 2**30, 1), "pool_blocks": eng.blocks.num_blocks, "pool_tokens": pool_tokens,
        "hbm_total_gib": round(torch.cuda.get_device_properties(0).total_memory / 2**30, 1),
        "weights_gib": round(eng.model.weight_bytes() / 2**30, 1),
        "decode_weight_layout": eng.decode_weight_layout,
        "working_set_tokens": distinct * a.prefix_len, "distinct_prefixes": distinct,
        "working_set_over_pool": round(distinct * a.prefix_len / pool_tokens, 2),
        "requests": len(reqs), "elapsed_s": round(el, 1), "req_per_s": round(len(reqs) / el, 2),
        "prompt_tok_per_s": round(prompt / el), "ttft_p50_ms": round(statistics.median(ttft), 1),
        "ttft_p99_ms": round(ttft[int(0.99 * len(ttft)) - 1], 1),
        "prefix_hit_tokens": hit, "prefix_hit_rate": round(hit / max(1, prompt), 4),
        "lru_evictions": kv["evictions"] - kv0["evictions"], "ttl_evictions": kv["ttl_evictions"] - kv0["ttl_evictions"],
        "cached_blocks_at_end": kv["cached"], "ttl_s": a.ttl, "zipf": a.zipf, "prefix_len": a.prefix_len,
        "suffix_len": a.suffix_len, "gen_len": a.gen_len, "concurrency": a.concurrency, "init_s": round(init_s, 1),
        "data": "synthetic token ids, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
