"""Prefill layer tail (o projection -> norm -> gate/up -> SiLU*mul -> down -> norm) at the bench's wave shape
(32 prompts x 512 tokens = 16,384 rows, Llama-3-8B), three ways:

  separate  o / down on hipBLASLt writing a fresh tensor, then fused_add_rms_norm (read h, read residual, write
            residual, write x: four [T, H] passes per norm)
  resid     o / down accumulate straight into the residual stream (``residual.addmm_``: hipBLASLt's beta = 1
            epilogue adds C = residual in fp32 before the single bf16 rounding), then a plain rms_norm (read
            residual, write x: two passes)
  resid+cN  as resid, the MLP run over N-row chunks so that the chunk's gate/up output (N x 28,672 bf16) and
            SiLU*mul output can stay in the 256 MB Infinity Cache between the three kernels

Median of 10 event-timed layer tails per variant; one JSON line each.

python bench/micro_prefill_tail.py [--tokens 16384] [--chunks 2048,4096]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--chunks", default="1024,2048,4096,8192")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t, h, i = a.tokens, a.hidden, a.inter
    bf = torch.bfloat16
    wo = (torch.randn(h, h, device=dev) * 0.02).to(bf)
    wgu = (torch.randn(2 * i, h, device=dev) * 0.02).to(bf)
    wd = (torch.randn(h, i, device=dev) * 0.02).to(bf)
    ones = torch.ones(h, dtype=bf, device=dev)
    attn = torch.randn(t, h, device=dev).to(bf)
    res0 = torch.randn(t, h, device=dev).to(bf)
    eps = 1e-5

    def separate(res):
        x = ops.fused_add_rms_norm(F.linear(attn, wo), res, ones, eps)
        hh = F.linear(ops.silu_and_mul(F.linear(x, wgu)), wd)
        return ops.fused_add_rms_norm(hh, res, ones, eps)

    def resid(res, chunk=0):
        res.addmm_(attn, wo.t())
        x = ops.rms_norm(res, ones, eps)
        if chunk <= 0 or chunk >= t:
            res.addmm_(ops.silu_and_mul(F.linear(x, wgu)), wd.t())
        else:
            gu = torch.empty(chunk, 2 * i, dtype=bf, device=dev)
            act = torch.empty(chunk, i, dtype=bf, device=dev)
            for s in range(0, t, chunk):
                e = min(t, s + chunk)
                n = e - s
                F.linear(x[s:e], wgu, out=gu[:n])
                ops.silu_and_mul(gu[:n], out=act[:n])
                res[s:e].addmm_(act[:n], wd.t())
        return ops.rms_norm(res, ones, eps)

    # numerics: the resid forms against the separate form (both bf16 GEMMs; resid rounds once instead of twice)
    r1, r2 = res0.clone(), res0.clone()
    y1, y2 = separate(r1), resid(r2)
    rel = ((r1.float() - r2.float()).norm() / r1.float().norm()).item()
    relx = ((y1.float() - y2.float()).norm() / y1.float().norm()).item()
    print(json.dumps({"check": "resid_vs_separate", "residual_rel_err": rel, "x_rel_err": relx}), flush=True)

    variants = [("separate", lambda r: separate(r))] + [("resid", lambda r: resid(r))]
    for c in [int(v) for v in a.chunks.split(",") if v]:
        variants.append((f"resid+c{c}", lambda r, c=c: resid(r, c)))
    flops = 2 * t * h * (h + 2 * i + i)
    for name, fn in variants:
        res = res0.clone()
        fn(res)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            res.copy_(res0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn(res)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        print(json.dumps({"variant": name, "tokens": t, "us_per_layer_tail": round(us, 1),
                          "gemm_TFps_equiv": round(flops / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
