#!/usr/bin/env python3
"""
Per-rank COMPUTE of a tensor-parallel configuration on ONE GPU (BASELINE config 4: Llama-3-70B TP=8):
rank 0's shard of the TP=N model (1/N of every projection, 8/N query heads and 1 KV head per rank at
70B TP=8, the vocab-parallel LM head slice) runs the bench's workload — waves of --batch requests,
--prompt-len → --gen-len tokens, hipGraph decode — with every collective replaced by a local
stand-in (src/parallel/tp.py ShardProbeTP). The printed times are what one rank of an N-GPU TP
group spends in kernels per prefill and per decode step; the all-reduces (2 per layer; 160 per 70B
decode step, 512 KiB each at batch 32) and the logits all-gather come on top and are NOT measured
here (one GPU). Tokens are meaningless (no real reduction); the timing is not.

    python bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1
"""

from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src import ops  # noqa: E402
from src.config import EngineConfig  # noqa: E402
from src.parallel.tp import ShardProbeTP  # noqa: E402
from src.parallel.tp_runner import build_tp_engine  # noqa: E402
from src.preproc import SamplingParams  # noqa: E402
from src.utils.tracing import prof_marker  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default="cuda:0", help="cpu: fp32 reference ops, for tests")
    ap.add_argument("--decode-window", type=int, default=8, help="EngineConfig.decode_window (1: single steps, A/B)")
    ap.add_argument("--legacy-fused", action="store_true",
                    help="A/B: round 5's fused-exchange rule (the table tile with its full LDS ring, zero slack)")
    ap.add_argument("--attn-static-parts", action="store_true",
                    help="A/B: decode attention split statically for few pairs too (ops.set_attn_few_pair_parts)")
    ap.add_argument("--max-model-len", type=int, default=0, help="engine bound (0: prompt + gen + 64)")
    a = ap.parse_args(argv)
    on_gpu = a.device.startswith("cuda")
    if a.attn_static_parts:
        ops.set_attn_few_pair_parts(False)
    mlen = a.max_model_len or a.prompt_len + a.gen_len + 64
    cfg = EngineConfig(max_num_seqs=a.batch, max_num_batched_tokens=max(16384, a.prompt_len), max_latency_ms=0.0,
                       graph_batch_sizes=sorted({1, 2, 4, 8, 16, 24, 32, a.batch}), decode_window=a.decode_window)
    t0 = time.perf_counter()
    tp = ShardProbeTP(a.tp)
    if a.legacy_fused:
        tp.fused_row_parallel = lambda n_tiles, grid=0, per_cu=0: True
    eng = build_tp_engine(a.preset, tp, a.device, cfg=cfg, max_model_len=mlen, seed=1234,
                          capture=on_gpu, dtype=torch.bfloat16 if on_gpu else torch.float32)
    eng.eos_token_id = None
    init_s = time.perf_counter() - t0
    rng = random.Random(5)
    vocab = eng.arch.vocab_size
    sp = SamplingParams(max_tokens=a.gen_len, ignore_eos=True)

    def wave():
        prompts = [[rng.randrange(3, vocab) for _ in range(a.prompt_len)] for _ in range(a.batch)]
        out = eng.generate(prompts, sp)
        assert all(len(o) == a.gen_len for o in out)

    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    for _ in range(a.warmup):
        wave()
    sync()
    prof_marker()
    s0 = dict(eng.stats)
    t1 = time.perf_counter()
    for _ in range(a.steps):
        wave()
    prof_marker()
    sync()
    el = time.perf_counter() - t1
    st = eng.stats
    dsteps = (a.gen_len - 1) * a.steps
    decode_ms = 1e3 * (st["decode_time"] - s0["decode_time"]) / dsteps
    prefill_ms = 1e3 * (st["prefill_time"] - s0["prefill_time"]) / a.steps
    wbytes = eng.runner.model.weight_bytes()
    print(json.dumps({
        "bench": "tp_shard_probe", "model": a.preset, "tp": a.tp, "rank": 0, "batch": a.batch,
        "decode_window": a.decode_window, "legacy_fused": a.legacy_fused,
        "prompt_len": a.prompt_len, "gen_len": a.gen_len, "dtype": "bf16" if on_gpu else "fp32", "weights": "random-init",
        "prefill_ms_per_wave": round(prefill_ms, 1), "decode_ms_per_step": round(decode_ms, 3),
        "wave_ms_compute_only": round(1e3 * el / a.steps, 1),
        "req_s_per_tp_group_compute_only": round(a.batch * a.steps / el, 2),
        "rank_weight_gib": round(wbytes / 2**30, 2), "engine_init_s": round(init_s, 1),
        "decode_windows": st.get("decode_windows", 0) - s0.get("decode_windows", 0),
        "queued_windows": st.get("queued_windows", 0) - s0.get("queued_windows", 0),
        "tp_fused": bool(eng.model.decode_plan(a.batch).get("tp_fused")),
        "o_tile": list(eng.model.decode_plan(a.batch)["o"]), "o_half_ring": eng.model.decode_plan(a.batch).get("o_half"),
        "down_tile": list(eng.model.decode_plan(a.batch)["down"] or []),
        "down_half_ring": eng.model.decode_plan(a.batch).get("down_half"),
        "not_included": "2 all-reduces per layer + the logits all-gather (one GPU: no peers)",
    }), flush=True)


if __name__ == "__main__":
    main()
