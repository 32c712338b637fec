"""
BASELINE config 5 — LLM workers behind ONE coordinator whose load balancer picks a worker per request — as a
reusable driver: the node section's ``lb_serving`` part (Mixtral-8x7B, one worker per GPU,
:func:`src.parallel.node_bench.lb_serving_part`) and the one-GPU rehearsal (``bench/lb_serving_bench.py``: several
worker processes sharing a GPU, one of them slower) both run :func:`serve_through_coordinator`.

The workload is config 5's: mixed prompt / output lengths whose prompts share Zipf-distributed prefixes (so the
workers' prefix caches hit, and — with their KV pools sized below the working set — evict, LRU among released
blocks plus the TTL), served closed-loop through the real path: client → coordinator (RPC) → ``least_latency``
(or another strategy) → worker (RPC) → continuous-batching engine. Reported: req/s, p50 / p99 latency, TTFT,
dispatches per worker, prefix-hit tokens and LRU / TTL evictions per worker (engine counters over the run).

Reference: `/root/reference/src/load_balancer.py:276-291` (least_latency),
`/root/reference/docs/router_vs_load_balancer.md:41-57`, `/root/reference/src/kvstore.py:82-102` (LRU).
"""

from __future__ import annotations

import asyncio
import random
import statistics
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple


@dataclass
class LBWorkload:
    requests: int = 256
    concurrency: int = 64
    prefixes: int = 24              # distinct shared prefixes
    zipf: float = 1.0
    prompt_min: int = 128
    prompt_max: int = 2048
    gen_choices: Tuple[int, ...] = (32, 64, 128, 256)
    seed: int = 0


def make_requests(w: LBWorkload, vocab: int) -> List[Dict[str, Any]]:
    """Token-id requests: a Zipf-chosen shared prefix (half to all of the prompt) + a private suffix; prompt lengths
    uniform in [prompt_min, prompt_max], outputs from gen_choices (ignore_eos: exactly that many tokens)."""
    rng = random.Random(w.seed)
    prefixes = [[rng.randrange(3, vocab) for _ in range(w.prompt_max)] for _ in range(w.prefixes)]
    weights = [1.0 / (i + 1) ** w.zipf for i in range(w.prefixes)]
    out = []
    for _ in range(w.requests):
        n = rng.randrange(w.prompt_min, w.prompt_max + 1)
        pre = rng.choices(prefixes, weights)[0][: rng.randrange(n // 2, n + 1)]
        ids = pre + [rng.randrange(3, vocab) for _ in range(n - len(pre))]
        out.append({"prompt_token_ids": ids, "max_tokens": rng.choice(w.gen_choices), "ignore_eos": True,
                    "return_text": False})
    return out


def _pct(xs: List[float], q: float) -> Optional[float]:
    if not xs:
        return None
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, max(0, int(round(q * len(xs))) - 1))], 2)


async def _engine_counters(rpc, addr: str, model: str) -> Dict[str, Any]:
    try:
        r = await rpc.call(addr, {"op": "engine_stats", "model": model}, timeout=30.0)
    except Exception:  # noqa: BLE001
        return {}
    st = (r or {}).get("stats") or {}
    kv = st.get("kv") or {}
    return {"prefix_hit_tokens": st.get("prefix_hit_tokens", 0), "prompt_tokens": st.get("prompt_tokens", 0),
            "generated_tokens": st.get("generated_tokens", 0), "finished": st.get("finished", 0),
            "lru_evictions": kv.get("evictions", 0), "ttl_evictions": kv.get("ttl_evictions", 0),
            "kv_blocks": kv.get("num_blocks"), "decode_weight_layout": st.get("decode_weight_layout")}


async def serve_through_coordinator(workers: Dict[str, str], model: str, arch: str, strategy: str,
                                    reqs: List[Dict[str, Any]], concurrency: int,
                                    health_interval_s: float = 1.0, warmup: Optional[List[Dict[str, Any]]] = None
                                    ) -> Dict[str, Any]:
    """Start a coordinator with ``strategy``, register every worker (id -> host:port) as a replica of ONE shard
    (the balancer chooses among all of them for every request), warm up, then drive ``reqs`` closed-loop with
    ``concurrency`` clients and report (see the module doc)."""
    from src.client import InferenceClient
    from src.coordinator import Coordinator
    from src.rpc import RPCClient

    coord = Coordinator(port=0, strategy=strategy, health_check_interval=health_interval_s,
                        request_timeout_s=1800.0)
    cport = await coord.start()
    rpc = RPCClient(max_idle_per_host=8)
    client = InferenceClient(f"127.0.0.1:{cport}", timeout=1800.0)
    try:
        for wid, addr in workers.items():
            coord.register_worker(wid, addr, {model: {"arch": arch}}, metadata={"shard_id": 0})
        from src.coordinator import DEFAULT_VERSION

        lb = coord._lb(model, DEFAULT_VERSION)
        for r in (warmup or []):  # one at a time per worker: graphs, hipBLASLt heuristics, first reports
            await client.infer(model, r, cache=False)
        before = {w: await _engine_counters(rpc, a, model) for w, a in workers.items()}
        disp0 = {w: lb.worker_stats[w].request_count for w in workers}
        lat: List[float] = []
        ttft: List[float] = []
        errors: List[str] = []
        nxt = [0]

        async def client_loop():
            while nxt[0] < len(reqs):
                i = nxt[0]
                nxt[0] += 1
                t0 = time.perf_counter()
                rep = await client.infer(model, reqs[i], cache=False)
                if not rep.get("success"):
                    errors.append(str(rep.get("error"))[:200])
                    continue
                o = rep.get("outputs") or {}
                if o.get("num_output_tokens") != reqs[i]["max_tokens"]:
                    errors.append(f"request {i}: {o.get('num_output_tokens')} tokens")
                lat.append((time.perf_counter() - t0) * 1e3)
                if o.get("ttft_ms") is not None:
                    ttft.append(float(o["ttft_ms"]))

        t0 = time.perf_counter()
        await asyncio.gather(*(client_loop() for _ in range(concurrency)))
        el = time.perf_counter() - t0
        after = {w: await _engine_counters(rpc, a, model) for w, a in workers.items()}
        per = {}
        for w in workers:
            b, a = before[w], after[w]
            per[w] = {"dispatched": lb.worker_stats[w].request_count - disp0[w],
                      **{k: (a.get(k, 0) or 0) - (b.get(k, 0) or 0) for k in
                         ("prefix_hit_tokens", "prompt_tokens", "generated_tokens", "lru_evictions", "ttl_evictions")},
                      "kv_blocks": a.get("kv_blocks"), "decode_weight_layout": a.get("decode_weight_layout")}
        hits = sum(p["prefix_hit_tokens"] for p in per.values())
        prompt = sum(p["prompt_tokens"] for p in per.values())
        return {"strategy": strategy, "requests": len(lat), "errors": errors[:5], "error_count": len(errors),
                "elapsed_s": round(el, 3), "req_s": round(len(lat) / el, 3) if el > 0 else None,
                "p50_latency_ms": _pct(lat, 0.5), "p99_latency_ms": _pct(lat, 0.99),
                "mean_latency_ms": round(statistics.mean(lat), 2) if lat else None,
                "ttft_p50_ms": _pct(ttft, 0.5), "ttft_p99_ms": _pct(ttft, 0.99),
                "prefix_hit_rate": round(hits / prompt, 4) if prompt else None,
                "lru_evictions": sum(p["lru_evictions"] for p in per.values()),
                "ttl_evictions": sum(p["ttl_evictions"] for p in per.values()),
                "per_worker": per}
    finally:
        client.close()
        rpc.close()
        await coord.stop()
