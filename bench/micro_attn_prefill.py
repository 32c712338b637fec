"""Prefill attention microbenchmark: 32 sequences x 512 new tokens (the bench's prefill), Llama-3-8B
geometry (32 q / 8 kv heads), paged KV; reports us per call and TFLOP/s (causal FLOPs)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402


def main():
    n, L = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (32, 512)
    dev = torch.device("cuda:0")
    hq, hkv, bs, d = 32, 8, 16, 128
    nb_seq = (L + bs - 1) // bs
    nblocks = n * nb_seq + 8
    kc = torch.randn(nblocks, hkv, bs, d, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nblocks, hkv, bs, d, device=dev, dtype=torch.bfloat16)
    # DIE_MICRO_BT=seq: blocks in allocation order (what a fresh engine hands out); default: a random permutation
    order = torch.arange(nblocks, device=dev) if os.environ.get("DIE_MICRO_BT") == "seq" else torch.randperm(nblocks, device=dev)
    bt = order[: n * nb_seq].view(n, nb_seq).to(torch.int32)
    cu = torch.arange(0, (n + 1) * L, L, dtype=torch.int32, device=dev)
    ctx = torch.full((n,), L, dtype=torch.int32, device=dev)
    q = torch.randn(n * L, (hq + 2 * hkv) * d, device=dev, dtype=torch.bfloat16)[:, : hq * d]
    out = torch.empty(n * L, hq * d, device=dev, dtype=torch.bfloat16)
    fn = lambda: ops.attn_prefill(q, kc, vc, bt, cu, ctx, L, hq, hkv, 1 / d ** 0.5, out=out)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 20
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / iters
    flop = 4 * n * hq * d * (L * (L + 1) / 2)
    print(json.dumps({"bench": "attn_prefill", "seqs": n, "len": L, "us": round(us, 1),
                      "TFLOPs": round(flop / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
