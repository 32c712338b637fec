"""Microbenchmark: paged decode attention (Llama-3-8B geometry: 32 q / 8 kv heads x 128).

Cold-cache protocol: the KV pool is ~4 GiB and the block tables are random permutations,
so KV bytes come from HBM as in a real decode step. Reports us per call and the effective
KV read bandwidth for the self-merging kernel (v3) and the two-launch path.
python bench/micro_attn_decode.py [batch] [ctx_lo] [ctx_hi]
"""
import json
import random
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from src import ops  # noqa: E402


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else 640
    dev = torch.device("cuda:0")
    hkv, g, bs, d = 8, 4, 16, 128
    hq = hkv * g
    nblocks = (4 << 30) // (2 * hkv * bs * d * 2)
    kc = torch.randn(nblocks, hkv, bs, d, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nblocks, hkv, bs, d, device=dev, dtype=torch.bfloat16)
    rng = random.Random(0)
    max_ctx = 8192
    for trial in range(3):
        ctxs = [rng.randint(lo, hi) for _ in range(b)]
        iters = 20  # every call reads its own blocks: 20 x ~75 MB >> the 256 MB Infinity Cache
        perms = [torch.randperm(nblocks, device=dev)[: b * (max_ctx // bs)].view(b, max_ctx // bs).to(torch.int32)
                 for _ in range(iters)]
        ctx = torch.tensor(ctxs, dtype=torch.int32, device=dev)
        q = torch.randn(b, (hq + 2 * hkv) * d, device=dev, dtype=torch.bfloat16)[:, : hq * d]
        maxp = ops.decode_partials(max_ctx)
        po = torch.empty(b * hq * maxp * d, dtype=torch.float32, device=dev)
        pm = torch.empty(b * hq * maxp * 2, dtype=torch.float32, device=dev)
        cnt = torch.zeros(b * hkv, dtype=torch.int32, device=dev)
        out = torch.empty(b, hq * d, dtype=torch.bfloat16, device=dev)
        kv_bytes = sum(ctxs) * hkv * d * 2 * 2
        for merge in (False, True):
            def fn(perm):
                ops.attn_decode(q, kc, vc, perm, ctx, max_ctx, hq, hkv, 0.088, part_o=po, part_ml=pm, out=out,
                                counters=cnt, merge_kernel=merge)
            fn(perms[0])
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for i in range(iters):
                    fn(perms[i])
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(5):
                s.record()
                gr.replay()
                e.record()
                torch.cuda.synchronize()
                best = min(best, s.elapsed_time(e) * 1e3 / iters)
            print(json.dumps({"bench": "attn_decode", "batch": b, "ctx": [lo, hi], "trial": trial,
                              "path": "two-launch" if merge else "v3", "us": round(best, 2),
                              "GBps": round(kv_bytes / best / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
