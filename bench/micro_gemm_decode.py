"""Microbenchmark: decode-shaped GEMMs (M = batch <= 32) — hipBLASLt (F.linear)
vs the hand-written weight-streaming kernel in every (mode, wr, sk) config.

Cold-cache protocol: the kernel cycles through enough distinct weight copies
(>= 1.5 GiB) that nothing is served from the 256 MiB Infinity Cache, as in the
real decode step where each layer's weights are read once. Prints one JSON
line per (shape, variant) with time per call and effective HBM GB/s."""

import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from src import ops  # noqa: E402

SHAPES = {  # name: (N_out, K, silu)
    "qkv_8b": (6144, 4096, False),
    "o_8b": (4096, 4096, False),
    "gate_up_8b": (14336, 4096, True),
    "down_8b": (4096, 14336, False),
    "lm_head_8b": (128256, 4096, False),
    "qkv_70b_tp8": (1280, 8192, False),
    "o_70b_tp8": (8192, 1024, False),
    "gate_up_70b_tp8": (3584, 8192, True),
    "down_70b_tp8": (8192, 3584, False),
}


def timeit(fn, ws, iters=None):
    n = len(ws)
    iters = iters or max(n, 8)
    for i in range(3):
        fn(ws[i % n])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(ws[i % n])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    if len(sys.argv) > 2 and sys.argv[2] == "nt":
        return main_nt(m)
    if len(sys.argv) > 2 and sys.argv[2] == "resid":
        return main_resid(m)
    if len(sys.argv) > 2 and sys.argv[2] == "warm":
        return main_warm(m)
    if len(sys.argv) > 2 and sys.argv[2] == "deep":
        return main_deep(m)
    if len(sys.argv) > 2 and sys.argv[2] == "moe":
        return main_moe(m)
    if len(sys.argv) > 2 and sys.argv[2] == "chain":
        return main_chain(m)
    dev = torch.device("cuda:0")
    for name, (n, k, silu) in SHAPES.items():
        wrows = 2 * n if silu else n
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        wbytes = wrows * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(wrows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        res = []
        if silu:
            res.append(("hipblaslt+silu", timeit(lambda w: ops.silu_and_mul(torch.nn.functional.linear(x, w)), ws)))
        else:
            res.append(("hipblaslt", timeit(lambda w: torch.nn.functional.linear(x, w), ws)))
        for wr in (32, 48, 64, 96, 112, 128):
            kc = 128 if wr >= 96 else 256
            if silu:
                if n % (wr // 2) == 0:
                    res.append((f"gd_silu_wr{wr}", timeit(lambda w: ops.gemm_decode(x, w, 1, wr, 1), ws)))
                continue
            if n % wr == 0:
                res.append((f"gd_bf16_wr{wr}", timeit(lambda w: ops.gemm_decode(x, w, 0, wr, 1), ws)))
            for sk in (2, 4, 8):
                if k % (kc * sk) == 0 and n % wr == 0 and (n // wr) * sk <= 1024:
                    res.append((f"gd_slab_wr{wr}_sk{sk}", timeit(lambda w: ops.gemm_decode(x, w, 2, wr, sk), ws)))
        for v, us in res:
            print(json.dumps({"shape": name, "M": m, "N": n, "K": k, "variant": v, "us": round(us, 2),
                              "GBps": round(wbytes / us / 1e3, 1)}), flush=True)
        del ws
        torch.cuda.empty_cache()


def main_nt(m):
    """Tuned config per shape, non-temporal vs default-policy weight loads."""
    dev = torch.device("cuda:0")
    for name, (n, k, silu) in SHAPES.items():
        if name.startswith("lm_head"):
            continue
        mode = 1 if silu else (0 if (n, k, 0) in ops.DECODE_GEMM_CFG else 2)
        wr, sk = ops._cfg_for(n, k, mode)
        wrows = 2 * n if silu else n
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        wbytes = wrows * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(wrows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        for nt in (False, True):
            us = timeit(lambda w: ops.gemm_decode(x, w, mode, wr, sk, nt=nt), ws)
            print(json.dumps({"shape": name, "M": m, "mode": mode, "wr": wr, "sk": sk, "nt": nt, "us": round(us, 2),
                              "GBps": round(wbytes / us / 1e3, 1)}), flush=True)
        del ws
        torch.cuda.empty_cache()



def main_resid(m):
    """Mode 3 (split-K + last-arriver residual update + norm statistics) tile sweep."""
    dev = torch.device("cuda:0")
    for name, (n, k) in {"o_8b": (4096, 4096), "down_8b": (4096, 14336)}.items():
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        wbytes = n * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(n, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        res = torch.randn(m, n, device=dev, dtype=torch.bfloat16)
        for wr in (32, 64, 128):
            for sk in (1, 2, 4, 8):
                kc = 128 if wr >= 96 else 256
                if k % (kc * sk) or (n // wr) * sk > 1024:
                    continue
                ssp = torch.zeros(n // wr, ops.SSP_LD, device=dev)
                cnt = torch.zeros(n // wr, dtype=torch.int32, device=dev)
                us = timeit(lambda w: ops.linear_slab_residual(x, w, res, ssp, cnt, wr, sk), ws)
                print(json.dumps({"shape": name, "M": m, "mode": 3, "wr": wr, "sk": sk, "us": round(us, 2),
                                  "GBps": round(wbytes / us / 1e3, 1)}), flush=True)
        del ws
        torch.cuda.empty_cache()


def main_warm(m):
    """Same weights every call (Infinity-Cache resident when they fit in 256 MB) vs cold copies:
    what a weight prefetch into the MALL could buy each decode projection."""
    dev = torch.device("cuda:0")
    for name, (n, k, silu) in SHAPES.items():
        if name.startswith("lm_head") or "70b" in name:
            continue
        mode = 1 if silu else 2
        wr, sk = ops._cfg_for(n, k, mode)
        wrows = 2 * n if silu else n
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        wbytes = wrows * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(wrows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        for nt in (True, False):
            cold = timeit(lambda w: ops.gemm_decode(x, w, mode, wr, sk, nt=nt), ws)
            warm = timeit(lambda w: ops.gemm_decode(x, w, mode, wr, sk, nt=nt), ws[:1], iters=max(8, copies))
            print(json.dumps({"shape": name, "MB": round(wbytes / 2**20, 1), "nt": nt, "cold_us": round(cold, 2),
                              "warm_us": round(warm, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


def main_deep(m):
    """Deep-ring variants (wr code rows+1: 128-wide K slots, 5-7 slots in flight) vs the tuned configs."""
    dev = torch.device("cuda:0")
    cand = {
        "qkv_8b": [(2, 48, 2), (2, 49, 2), (2, 49, 4), (2, 65, 2), (2, 65, 4), (2, 33, 2)],
        "o_8b": [(2, 64, 4), (2, 65, 4), (2, 65, 2), (2, 33, 2), (2, 49, 4)],
        "gate_up_8b": [(1, 112, 1), (1, 65, 1), (1, 33, 1), (1, 64, 1)],
        "down_8b": [(2, 64, 4), (2, 65, 4), (2, 65, 2), (2, 33, 2), (2, 49, 4)],
        "lm_head_8b": [(0, 64, 1), (0, 65, 1)],
    }
    for name, cfgs in cand.items():
        n, k, silu = SHAPES[name]
        wrows = 2 * n if silu else n
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        wbytes = wrows * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(wrows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        for mode, wr, sk in cfgs:
            us = timeit(lambda w: ops.gemm_decode(x, w, mode, wr, sk), ws)
            print(json.dumps({"shape": name, "mode": mode, "wr": wr, "sk": sk, "us": round(us, 2),
                              "GBps": round(wbytes / us / 1e3, 1)}), flush=True)
        del ws
        torch.cuda.empty_cache()



def main_moe(m):
    """Activation-image height A/B (run under DIE_GD_XR16=0 and =1): the tuned dense configs at M = m,
    and Mixtral-8x7B's grouped expert projections at m tokens, top-2 random routing."""
    dev = torch.device("cuda:0")
    xr16 = __import__("os").environ.get("DIE_GD_XR16", "1")
    for name in ("qkv_8b", "o_8b", "gate_up_8b", "down_8b"):
        n, k, silu = SHAPES[name]
        mode = 1 if silu else (0 if (n, k, 0) in ops.DECODE_GEMM_CFG else 2)
        wr, sk = ops._cfg_for(n, k, mode)
        wrows = 2 * n if silu else n
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        wbytes = wrows * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(wrows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        us = timeit(lambda w: ops.gemm_decode(x, w, mode, wr, sk), ws)
        print(json.dumps({"shape": name, "M": m, "xr16": xr16, "us": round(us, 2),
                          "GBps": round(wbytes / us / 1e3, 1)}), flush=True)
        del ws
    e, h, inter = 8, 4096, 14336
    ids = torch.stack([torch.randperm(e, device=dev)[:2] for _ in range(m)]).to(torch.int32)
    offsets, sorted_idx, pos = ops.moe_align(ids, e)
    xs = torch.randn(2 * m, h, device=dev, dtype=torch.bfloat16)
    a = torch.empty(2 * m, inter, device=dev, dtype=torch.bfloat16)
    ys = torch.empty(2 * m, h, device=dev, dtype=torch.bfloat16)
    w13s = [torch.randn(e, 2 * inter, h, device=dev, dtype=torch.bfloat16) / 64 for _ in range(2)]
    w2s = [torch.randn(e, h, inter, device=dev, dtype=torch.bfloat16) / 64 for _ in range(2)]
    kern = ops._kern()
    none = torch.empty(0, dtype=torch.int32, device=dev)
    wr1 = ops._cfg_for(inter, h, 1)[0]
    wr2 = ops._moe_down_wr(h, inter)
    for nm, ws, fn in (("moe_w13", w13s, lambda w: kern.gemm_decode_grouped(a, xs, w, offsets, 1, *ops.gd_tile(wr1),
                                                                            none, 1, m, 1)),
                       ("moe_w2", w2s, lambda w: kern.gemm_decode_grouped(ys, a, w, offsets, 0, *ops.gd_tile(wr2),
                                                                          none, 1, m, 1))):
        us = timeit(fn, ws)
        wbytes = ws[0].numel() * 2
        print(json.dumps({"shape": nm, "M": m, "rows_per_expert": (offsets[1:] - offsets[:-1]).tolist(),
                          "xr16": xr16, "us": round(us, 2), "GBps": round(wbytes / us / 1e3, 1)}), flush=True)


def main_chain(m):
    """What one launch streaming n gate/up-sized weight sets back to back (grouped kernel, every expert
    gets all m rows) buys over n dense launches: the per-launch fill/drain/straggler cost that a
    persistent decode layer would remove. Cold weights (8 copies cycled)."""
    dev = torch.device("cuda:0")
    kern = ops._kern()
    h, inter = 4096, 14336
    wr = ops._cfg_for(inter, h, 1)[0]
    x = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    none = torch.empty(0, dtype=torch.int32, device=dev)
    for n in (1, 2, 4, 8):
        ws = [torch.randn(n, 2 * inter, h, device=dev, dtype=torch.bfloat16) / 64 for _ in range(max(2, 8 // n))]
        xs = x.repeat(n, 1).contiguous()
        a = torch.empty(n * m, inter, device=dev, dtype=torch.bfloat16)
        offsets = torch.arange(0, (n + 1) * m, m, dtype=torch.int32, device=dev)
        one = timeit(lambda w: kern.gemm_decode_grouped(a, xs, w, offsets, 1, *ops.gd_tile(wr), none, 1, m, 1), ws)
        sep = timeit(lambda w: [ops.gemm_decode(x, w[i], 1, wr, 1) for i in range(n)], ws)
        wbytes = n * 2 * inter * h * 2
        print(json.dumps({"bench": "chain", "M": m, "n_weight_sets": n, "one_launch_us": round(one, 2),
                          "separate_launches_us": round(sep, 2), "one_launch_TBps": round(wbytes / one / 1e6, 2),
                          "separate_TBps": round(wbytes / sep / 1e6, 2)}), flush=True)
        del ws

if __name__ == "__main__":
    main()
