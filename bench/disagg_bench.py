#!/usr/bin/env python3
"""
BASELINE config 3: Llama-3-8B disaggregated serving — a prefill engine computes each prompt's KV
and first token, the packed KV blocks are shipped to a decode engine, which joins them to its
continuous decode batch without recomputing the prompt (src/engine/disagg.py).

With two visible GPUs the prefill engine runs on cuda:0 and the decode engine on cuda:1 (the KV
moves GPU→GPU over xGMI, hipMemcpyPeerAsync on a transfer stream). On a one-GPU box both engines
share cuda:0 (and its weights): the numbers then show the protocol's cost against colocated
serving (bench.py), not the two-GPU pipeline's gain.

One step = a wave of --batch requests (random --prompt-len prompts, --gen-len tokens, greedy,
ignore_eos) submitted together and served to completion. Prints one JSON line.

    python bench/disagg_bench.py --steps 3 --warmup 1
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.config import EngineConfig  # noqa: E402
from src.engine import LLMEngine  # noqa: E402
from src.engine.async_engine import AsyncLLMEngine  # noqa: E402
from src.engine.disagg import DisaggregatedServer  # noqa: E402
from src.preproc import SamplingParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--kv-blocks", type=int, default=4096)
    a = ap.parse_args()
    two = torch.cuda.device_count() >= 2
    dp, dd = torch.device("cuda:0"), torch.device("cuda:1" if two else "cuda:0")
    mlen = a.prompt_len + a.gen_len + 64
    cfg = EngineConfig(max_num_seqs=a.batch, max_num_batched_tokens=max(16384, a.prompt_len), max_latency_ms=0.0,
                       num_kv_blocks=a.kv_blocks, graph_batch_sizes=[1, 2, 4, 8, 16, 24, 32, a.batch])
    t_init = time.perf_counter()
    pre = LLMEngine.from_preset(a.preset, device=dp, cfg=cfg, max_model_len=mlen, seed=1234, capture=False)
    if two:
        dec = LLMEngine.from_preset(a.preset, device=dd, cfg=cfg, max_model_len=mlen, seed=1234, capture=True)
    else:  # same GPU: share the weights, own KV pool and decode graphs
        dec = LLMEngine(pre.model, cfg, mlen)
        dec.runner.capture_graphs()
    for e in (pre, dec):
        e.eos_token_id = None
    init_s = time.perf_counter() - t_init
    srv = DisaggregatedServer(AsyncLLMEngine(pre, "prefill"), AsyncLLMEngine(dec, "decode"))
    rng = random.Random(7)
    vocab = pre.arch.vocab_size

    async def wave():
        prompts = [[rng.randrange(3, vocab) for _ in range(a.prompt_len)] for _ in range(a.batch)]
        sp = SamplingParams(max_tokens=a.gen_len, ignore_eos=True)

        async def one(p):
            t0 = time.perf_counter()
            s = await srv.generate(p, sp)
            assert len(s.output_ids) == a.gen_len, len(s.output_ids)
            return time.perf_counter() - t0

        return await asyncio.gather(*(one(p) for p in prompts))

    async def run():
        srv.start()
        try:
            for _ in range(a.warmup):
                await wave()
            torch.cuda.synchronize()
            b0 = srv.bytes_moved
            t0 = time.perf_counter()
            lats = []
            for _ in range(a.steps):
                lats += await wave()
            torch.cuda.synchronize()
            return time.perf_counter() - t0, lats, srv.bytes_moved - b0
        finally:
            srv.stop()

    el, lats, moved = asyncio.run(run())
    n = a.steps * a.batch
    print(json.dumps({
        "bench": "disaggregated", "config": "BASELINE 3", "model": a.preset, "gpus": 2 if two else 1,
        "topology": "prefill cuda:0 -> decode cuda:1 (xGMI)" if two else "prefill and decode engines share cuda:0",
        "req_s": round(n / el, 3), "p50_latency_ms": round(1e3 * statistics.median(lats), 1),
        "ms_per_wave": round(1e3 * el / a.steps, 1), "kv_moved_gib": round(moved / 2**30, 2),
        "kv_gib_per_s": round(moved / 2**30 / el, 1), "batch": a.batch, "prompt_len": a.prompt_len,
        "gen_len": a.gen_len, "engine_init_s": round(init_s, 1), "weights": "random-init", "dtype": "bf16",
    }), flush=True)


if __name__ == "__main__":
    main()
