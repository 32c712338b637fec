"""Serving stress test: mixed prompt lengths, generation lengths and sampling settings, with
shared prefixes and a small KV pool (forces prefix-cache eviction and preemption), through
client -> coordinator -> worker. Every request must succeed with the requested token count.

python bench/stress.py [--preset llama-mini] [--requests 400] [--concurrency 64] [--kv-blocks 600]
"""
import argparse
import asyncio
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.client import InferenceClient  # noqa: E402
from src.config import ModelConfig  # noqa: E402
from src.coordinator import Coordinator  # noqa: E402
from src.worker import Worker  # noqa: E402


async def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama-mini")
    ap.add_argument("--requests", type=int, default=400)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--kv-blocks", type=int, default=600)
    ap.add_argument("--max-model-len", type=int, default=2048)
    ap.add_argument("--text-frac", type=float, default=0.0, help="share of requests sent as text prompts")
    ap.add_argument("--preproc-processes", type=int, default=0, help="tokenise / detokenise text out of process")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    cfg = ModelConfig(model_name="m", model_path="", arch="llama", preset=a.preset, max_batch_size=32,
                      max_model_len=a.max_model_len, max_num_batched_tokens=4096, num_kv_blocks=a.kv_blocks,
                      use_cuda_graph=True, max_latency_ms=5.0, overrides={"device": "cuda:0"},
                      preproc_processes=a.preproc_processes)
    w = Worker("s0", host="127.0.0.1", install_signal_handlers=False)
    assert w.load_model(cfg)
    wport = await w.start()
    coord = Coordinator(port=0, max_batch_size=32, max_latency_ms=5)
    cport = await coord.start()
    await coord.add_static_worker(f"127.0.0.1:{wport}")
    c = InferenceClient(f"127.0.0.1:{cport}")
    rng = random.Random(a.seed)
    prefixes = [[rng.randrange(3, 30000) for _ in range(rng.randrange(16, 400))] for _ in range(6)]
    reqs = []
    for i in range(a.requests):
        body = prefixes[rng.randrange(6)] if rng.random() < 0.5 else []
        body = body + [rng.randrange(3, 30000) for _ in range(rng.randrange(1, 900))]
        mt = rng.choice([1, 2, 7, 16, 64, 200])
        mt = max(1, min(mt, a.max_model_len - len(body) - 1))
        r = {"prompt_token_ids": body, "max_tokens": mt, "ignore_eos": True}
        if rng.random() < a.text_frac:  # a text prompt of about the same length (byte tokenizer: 1 token per byte)
            r = {"prompt": "".join(chr(97 + rng.randrange(26)) for _ in range(max(1, min(len(body), 900)))),
                 "max_tokens": mt, "ignore_eos": True}
        if rng.random() < 0.4:
            r.update(temperature=rng.choice([0.7, 1.0]), top_k=rng.choice([0, 20]), top_p=rng.choice([1.0, 0.9]),
                     seed=i)
        reqs.append(r)
    sem = asyncio.Semaphore(a.concurrency)
    bad, lat = [], []

    async def one(i, r):
        async with sem:
            t0 = time.perf_counter()
            res = await c.infer("m", r, cache=False)
            lat.append(time.perf_counter() - t0)
            if not res.get("success") or res["outputs"]["num_output_tokens"] != r["max_tokens"] or \
                    ("prompt" in r and not isinstance(res["outputs"].get("text"), str)):
                bad.append((i, str(res)[:300]))

    t0 = time.perf_counter()
    await asyncio.wait_for(asyncio.gather(*(one(i, r) for i, r in enumerate(reqs))), 1800)
    el = time.perf_counter() - t0
    st = await InferenceClient(f"127.0.0.1:{wport}").call({"op": "engine_stats", "model": "m"})
    kv = st["stats"].get("kv") or {}
    backend = w.models["m"]
    print(json.dumps({"bench": "stress", "preset": a.preset, "requests": a.requests, "failed": len(bad),
                      "elapsed_s": round(el, 1), "req_per_s": round(a.requests / el, 1),
                      "text_requests": sum(1 for r in reqs if "prompt" in r),
                      "kv_blocks_used_after": kv.get("used"), "kv_evictions": kv.get("evictions"),
                      "preproc": backend.preproc.stats() if backend.preproc is not None else None,
                      "engine": {k: st["stats"].get(k) for k in ("preemptions", "swaps_out", "prefix_hit_tokens", "steps",
                                                                 "decode_windows", "generated_tokens")}}),
          flush=True)
    if kv.get("used"):
        bad.append(("kv", f"{kv.get('used')} KV blocks still held after every request finished"))
    for b in bad[:5]:
        print("FAILED", b, flush=True)
    c.close()
    await coord.stop()
    await w.shutdown()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    asyncio.run(main())
