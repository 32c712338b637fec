"""Open-loop serving benchmark: Poisson arrivals into one GPU engine.

The headline bench (bench.py) submits synchronized waves, which cannot show what per-iteration
admission buys. Here requests arrive one by one at exponential inter-arrival times (fixed seed) and
are served by the continuous-batching engine (AsyncLLMEngine thread, hipGraph decode, mixed steps):

* TTFT   — submit -> first token (client side);
* TPOT   — (last token - first token) / (n - 1) per request: the decode-interval a user sees;
* e2e    — submit -> last token;
* p50 / p99 of each, per arrival rate, for each ``mixed_batching`` policy (auto / always / off).

The reference's admission is the Batcher's size-or-latency flush (`/root/reference/src/batcher.py:144-166`);
prefill-only steps are the same flush at iteration granularity, mixed steps its continuous form.

    python bench/poisson_bench.py --rates 10,20,30,40 --requests 200
Prints one JSON line per (mode, rate), plus the pure-decode step time measured on a closed wave.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from src.config import EngineConfig  # noqa: E402
from src.engine import LLMEngine  # noqa: E402
from src.engine.async_engine import AsyncLLMEngine  # noqa: E402
from src.preproc import SamplingParams  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, max(0, int(round(q / 100 * len(xs))) - 1))]


async def run_rate(aeng, rate, n, prompt_len, gen_len, vocab, seed):
    rng = random.Random(seed)
    prompts = [[rng.randrange(3, vocab) for _ in range(prompt_len)] for _ in range(n)]
    gaps = [rng.expovariate(rate) for _ in range(n)]
    loop = asyncio.get_running_loop()
    rec = []

    async def one(i, t_sub):
        toks = []
        fut = aeng.submit(f"p{seed}-{i}", prompts[i], SamplingParams(max_tokens=gen_len, ignore_eos=True), loop,
                          on_token=lambda tok: toks.append(time.perf_counter()))
        seq = await fut
        t_end = time.perf_counter()
        assert len(seq.output_ids) == gen_len, (len(seq.output_ids), seq.finish_reason)
        rec.append((t_sub, toks[0], toks[-1], t_end, len(toks)))

    tasks = []
    t0 = time.perf_counter()
    t_next = t0
    for i in range(n):
        t_next += gaps[i]
        d = t_next - time.perf_counter()
        if d > 0:
            await asyncio.sleep(d)
        tasks.append(asyncio.ensure_future(one(i, time.perf_counter())))
    await asyncio.gather(*tasks)
    span = time.perf_counter() - t0
    ttft = [(a - s) * 1e3 for s, a, _, _, _ in rec]
    tpot = [(b - a) * 1e3 / max(1, k - 1) for _, a, b, _, k in rec]
    e2e = [(e - s) * 1e3 for s, _, _, e, _ in rec]
    return {"achieved_rps": round(n / span, 2),
            "ttft_ms": {"p50": round(pct(ttft, 50), 1), "p99": round(pct(ttft, 99), 1)},
            "tpot_ms": {"p50": round(pct(tpot, 50), 2), "p99": round(pct(tpot, 99), 2),
                        "mean": round(statistics.mean(tpot), 2)},
            "e2e_ms": {"p50": round(pct(e2e, 50), 1), "p99": round(pct(e2e, 99), 1)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--rates", default="10,20,30,40")
    ap.add_argument("--requests", type=int, default=200)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--max-num-seqs", type=int, default=64)
    ap.add_argument("--mixed-step-tokens", type=int, default=64)
    ap.add_argument("--modes", default="auto,off,always")
    # prefill batching under load, "tokens:wait_ms" per run (0:0 = off; EngineConfig.prefill_batch_tokens)
    ap.add_argument("--prefill-batch", default="0:0")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    dev = torch.device("cuda:0" if a.device == "cuda" else "cpu")
    cfg = EngineConfig(max_num_seqs=a.max_num_seqs, max_num_batched_tokens=16384, max_latency_ms=0.0,
                       mixed_step_tokens=a.mixed_step_tokens)
    kw = {} if a.device == "cuda" else {"capture": False, "dtype": torch.float32}
    eng = LLMEngine.from_preset(a.preset, device=dev, cfg=cfg, max_model_len=2048, seed=1234, **kw)
    eng.eos_token_id = None
    vocab = eng.arch.vocab_size
    aeng = AsyncLLMEngine(eng)
    aeng.start()

    async def closed_wave(n):
        rng = random.Random(5)
        ps = [[rng.randrange(3, vocab) for _ in range(a.prompt_len)] for _ in range(n)]
        futs = [aeng.submit(f"w{i}-{time.monotonic_ns()}", p, SamplingParams(max_tokens=a.gen_len, ignore_eos=True))
                for i, p in enumerate(ps)]
        await asyncio.gather(*futs)

    async def go():
        await closed_wave(32)  # warm-up (graphs, allocator, hipBLASLt)
        s0 = dict(eng.stats)
        await closed_wave(32)
        dstep = (eng.stats["decode_time"] - s0["decode_time"]) / (a.gen_len - 1) * 1e3
        print(json.dumps({"bench": "poisson", "pure_decode_step_ms_batch32": round(dstep, 3)}), flush=True)
        runs = [(mode, pb) for mode in a.modes.split(",") for pb in a.prefill_batch.split(",")]
        for mi, (mode, pb) in enumerate(runs):
            eng.cfg.mixed_batching = mode
            pbt, pbw = pb.split(":")
            eng.cfg.prefill_batch_tokens, eng.cfg.prefill_batch_wait_ms = int(pbt), float(pbw)
            for r in (float(x) for x in a.rates.split(",")):
                st0 = dict(eng.scheduler.stats())
                hit0 = eng.stats["prefix_hit_tokens"]
                t0s = {k: eng.stats.get(k, 0.0) for k in ("prefill_time", "decode_time", "mixed_time")}
                # distinct prompts per (mode, rate): no run is served from another run's cached prefix blocks
                res = await run_rate(aeng, r, a.requests, a.prompt_len, a.gen_len, vocab, seed=int(r * 100) + 7919 * mi)
                res["prefix_hit_tokens"] = eng.stats["prefix_hit_tokens"] - hit0
                st1 = eng.scheduler.stats()
                steps = {k: st1[k] - st0[k] for k in ("steps_prefill", "steps_decode", "steps_mixed")}
                # engine time per step kind (decode steps counted per scheduler step: a window of k steps is one)
                res["ms_per_step"] = {k.split("_")[0]: round((eng.stats.get(k, 0.0) - t0s[k]) * 1e3 / max(1, steps[n]), 2)
                                      for k, n in (("prefill_time", "steps_prefill"), ("decode_time", "steps_decode"),
                                                   ("mixed_time", "steps_mixed"))}
                res.update({"bench": "poisson", "mode": mode, "prefill_batch": {"tokens": int(pbt), "wait_ms": float(pbw)},
                            "rate_rps": r, "requests": a.requests,
                            "model": a.preset, "prompt_len": a.prompt_len, "gen_len": a.gen_len,
                            "tpot_p99_over_decode_step": round(res["tpot_ms"]["p99"] / dstep, 3), "steps": steps})
                print(json.dumps(res), flush=True)

    try:
        asyncio.run(go())
    finally:
        aeng.stop()


if __name__ == "__main__":
    main()
