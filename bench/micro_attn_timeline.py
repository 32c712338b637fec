"""Diagnostic: per-workgroup phase timeline of the fused decode attention (attn_decode_v3_kernel,
FUSED prologue) — by default the headline shape, 32 sequences x 8 kv heads (Llama-3-8B: 32 q heads x 128),
contexts 512..640; ``--shape 70b_tp8`` is a Llama-3-70B TP=8 rank (1 kv head, 8 q heads), ``--ctx N`` gives
every sequence the same context (as in a bench wave), ``--max-ctx`` the static bound that sizes the parts
(C = chunks per task). KV blocks allocated contiguously per sequence as the engine's block manager does, cold
KV (a new pool slice per call). Stamps (s_memrealtime, 100 MHz): entry, first chunk landed, prologue done,
stream done, end. Prints the median phase durations, the kernel span and the event-timed us per call."""

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402
from src.ops import reference as ref  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8b", choices=["8b", "70b_tp8", "8b_tp2"])
    ap.add_argument("--ctx", type=int, default=0, help="every sequence's context (0: 512 + 4 i)")
    ap.add_argument("--max-ctx", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--static-parts", action="store_true", help="A/B: the static split also for few pairs")
    ap.add_argument("--sk", type=int, default=0, help="qkv split-K slabs the prologue sums (0: the engine's tile)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n, bs, d = a.batch, 16, 128
    hkv, g, hid = {"8b": (8, 4, 4096), "70b_tp8": (1, 8, 8192), "8b_tp2": (4, 4, 4096)}[a.shape]
    hq = hkv * g
    ctxs = [a.ctx] * n if a.ctx else [512 + 4 * i for i in range(n)]
    max_ctx = a.max_ctx
    per_seq = max_ctx // bs
    copies = 12 if a.shape == "8b" else 40         # >> the 256 MB Infinity Cache
    nb = copies * n * per_seq
    kc = torch.randn(nb, hkv, bs, d, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nb, hkv, bs, d, device=dev, dtype=torch.bfloat16)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=dev)
    bts = [torch.arange(c * n * per_seq, (c + 1) * n * per_seq, device=dev, dtype=torch.int32).view(n, per_seq)
           for c in range(copies)]
    width = (hq + 2 * hkv) * d
    sk = a.sk or ops.decode_tile(width, hid, 2, max_sk=max(1, 50 // (g + 2)))[2]  # as CausalLM picks it
    slab = torch.randn(sk, n, width, device=dev) * 0.7
    ssp = torch.zeros(hid // 64, ops.SSP_LD, device=dev)
    ssp[:, :n] = float(hid) / ssp.shape[0]
    pos = (ctx - 1).long()
    cs = ref.rope_cos_sin(8192, d, 500000.0, dev)
    maxp = ops.decode_partials(max_ctx)
    po = torch.empty(n * hq * maxp * d, device=dev)
    pm = torch.empty(n * hq * maxp * 2, device=dev)
    cnt = torch.zeros(n * hkv, dtype=torch.int32, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ts = torch.zeros(copies, 2 * ncu * 6, dtype=torch.int64, device=dev)  # grids of up to 2 workgroups per CU
    kv_bytes = sum(ctxs) * hkv * d * 2 * 2

    def call(c):
        slots = (bts[c][torch.arange(n, device=dev), (ctx - 1).long() // bs].long() * bs + (ctx - 1).long() % bs)
        ops.attn_decode_fused(slab, ssp, pos, cs, slots, kc, vc, bts[c], ctx, max_ctx, hq, hkv, d ** -0.5, 1e-5, hid,
                              po, pm, cnt)

    for c in range(copies):
        call(c)
    torch.cuda.synchronize()
    k_ = ops._kern()
    k_.attn_set_few_pair_parts(not a.static_parts)
    for c in range(copies):
        k_.attn_set_timestamps(ts[c])
        call(c)
    k_.attn_set_timestamps(torch.empty(0, dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 3
    for _ in range(reps):
        for c in range(copies):
            call(c)
    e1.record()
    torch.cuda.synchronize()
    us_call = e0.elapsed_time(e1) * 1e3 / (reps * copies)
    t = ts.view(copies, 2 * ncu, 6).cpu().double()
    res = {k: [] for k in ("span", "first_chunk", "prologue", "stream", "merge_out", "start_skew", "tail")}
    for c in range(2, copies):
        tt = t[c]
        used = tt[:, 3] > 0  # workgroups that ran a task (a tensor-parallel shard leaves some without one)
        tt = tt[used]
        t0 = tt[:, 0].min()
        res["span"].append(float(tt[:, 4].max() - t0) * 10e-3)
        res["start_skew"].append(float(tt[:, 0].max() - t0) * 10e-3)
        res["tail"].append(float(tt[:, 4].max() - tt[:, 4].median()) * 10e-3)
        res["first_chunk"].append(float((tt[:, 1] - tt[:, 0]).median()) * 10e-3)
        res["prologue"].append(float((tt[:, 2] - tt[:, 1]).median()) * 10e-3)
        res["stream"].append(float((tt[:, 3] - tt[:, 2]).median()) * 10e-3)
        res["merge_out"].append(float((tt[:, 4] - tt[:, 3]).median()) * 10e-3)
    out = {k: round(statistics.median(v), 2) for k, v in res.items()}
    out["kv_TBps_span"] = round(kv_bytes / out["span"] / 1e6, 2)
    out["us_per_call"] = round(us_call, 2)
    out["kv_TBps_call"] = round(kv_bytes / us_call / 1e6, 2)
    print(json.dumps({"bench": "attn_decode_timeline", "shape": a.shape, "batch": n, "ctx": [ctxs[0], ctxs[-1]],
                      "max_ctx": max_ctx, "qkv_sk": sk, "workgroups_with_a_task": int((t[-1][:, 3] > 0).sum()),
                      **out}), flush=True)


if __name__ == "__main__":
    main()
