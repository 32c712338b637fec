"""Decode-GEMM tile sweep at tensor-parallel shard shapes (32 rows, tile-order weights, cold: a 1 GiB buffer is
written before every call; median of 10 event-timed calls). For each projection of a TP rank's decode layer —
qkv (mode 2: fp32 split-K slabs), o / down (mode 3: split-K + last-arriver residual update, the local form of the
fused row-parallel exchange) and gate/up (mode 4 full-K / mode 6 split-K, norm row scale + SiLU) — every valid
(wr, kc, sk) tile is timed. One JSON line per (shape, tile); the fastest per shape goes into ops.DECODE_TILE_CFG /
DECODE_SILU_SPLITK_CFG.

python bench/micro_tp_tiles.py [--shapes 70b_tp8,8b_tp2]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src import ops  # noqa: E402

SHAPES = {  # name -> [(projection, N, K, modes)]
    "70b_tp8": [("qkv", 1280, 8192, (2,)), ("o", 8192, 1024, (3,)), ("gate_up", 3584, 8192, (4, 6)),
                ("down", 8192, 3584, (3,))],
    "8b_tp2": [("qkv", 3072, 4096, (2,)), ("o", 4096, 2048, (3,)), ("gate_up", 7168, 4096, (4, 6)),
               ("down", 4096, 7168, (3,))],
    "8b": [("qkv", 6144, 4096, (2,)), ("o", 4096, 4096, (3,)), ("gate_up", 14336, 4096, (4, 6)),
           ("down", 4096, 14336, (3,))],
    "8b_tp4": [("qkv", 1536, 4096, (2,)), ("o", 4096, 1024, (3,)), ("gate_up", 3584, 4096, (4, 6)),
               ("down", 4096, 3584, (3,))],
    # Llama-3-70B on ONE GPU (TP=1): its tile-order copies do not fit beside 141 GB of weights, so decode streams the
    # row-major weights (--row-major)
    "70b": [("qkv", 10240, 8192, (2,)), ("o", 8192, 8192, (3,)), ("gate_up", 28672, 8192, (4, 6)),
            ("down", 8192, 28672, (3,))],
    # the decode step's LM head (Llama-3 vocabulary): mode 0, bf16 logits; row-major weight ("tiled": False)
    # as the engine stores it today, and tile-order
    "lm_head": [("lm_head", 128256, 4096, (0,))],
}
TILES = [(32, 256), (48, 256), (64, 256), (32, 128), (48, 128), (64, 128), (96, 128), (112, 128), (128, 128),
         (64, 64), (128, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="70b_tp8,8b_tp2")
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--proj", default="", help="comma-separated projections to sweep (default: all)")
    ap.add_argument("--splits", default="1,2,4,8", help="split-K counts to try (uneven splits allowed: 3,5,6)")
    ap.add_argument("--row-major", action="store_true", help="time the row-major weights (no tile-order copy)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    kern = ops._kern()
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    e = torch.empty(0, device=dev)
    m = a.rows
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for sname in a.shapes.split(","):
        for proj, n, k, modes in SHAPES[sname]:
            if a.proj and proj not in a.proj.split(","):
                continue
            silu = proj == "gate_up"
            w = (torch.randn(2 * n if silu else n, k, device=dev) * 0.02).to(torch.bfloat16)
            x = torch.randn(m, k, device=dev).to(torch.bfloat16)
            ssp = (torch.rand(4, 128, device=dev) * k * 0.1).float()
            best = None
            for mode in modes:
                sks = (1,) if mode == 4 else tuple(int(v) for v in a.splits.split(","))
                for (wr, kc), tiled in ([(t, False) for t in TILES] if a.row_major else
                                        [(t, True) for t in TILES] + ([(t, False) for t in TILES]
                                                                      if proj == "lm_head" else [])):
                    for sk in sks:
                        cols = wr // 2 if silu else wr
                        if n % cols or k % kc or k // kc < sk or not ops.gd_tile_valid(wr, kc, 32):
                            continue
                        lim = ops.SSP_MAX_TILES if m <= 32 else ops.SSP_MAX_TILES_WIDE
                        if mode == 3 and (wr not in (32, 64, 128) or n // wr > lim):
                            continue  # the fused path's consumers take <= 256 (<= 128 above 32 rows) tiles
                        if mode == 6 and sk == 1:
                            continue
                        ntiles = n // cols
                        if ntiles * sk > 4 * cus and proj != "lm_head":
                            continue
                        if mode == 0 and sk > 1:
                            continue
                        try:
                            wt = ops.gd_pack_weights(w, wr, silu=silu, kc=kc) if tiled else w
                        except AssertionError:
                            continue
                        cnt = torch.zeros(max(1, ntiles), dtype=torch.int32, device=dev)
                        tb = 32 if tiled else 0
                        if mode == 0:
                            y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
                            args = (y, x, wt, tb, wr, kc, 1, True, e, e, e, e, 0.0)
                        elif mode == 2:
                            y = torch.empty(sk, m, n, dtype=torch.float32, device=dev)
                            args = (y, x, wt, 2 | tb, wr, kc, sk, True, e, e, e, e, 0.0)
                        elif mode == 3:
                            y = torch.empty(sk, m, n, dtype=torch.float32, device=dev)
                            resid = torch.zeros(m, n, dtype=torch.bfloat16, device=dev)
                            sspo = torch.zeros(ntiles, 128, device=dev)
                            args = (y, x, wt, 3 | tb, wr, kc, sk, True, resid, sspo, cnt, e, 0.0)
                        else:
                            y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
                            slab = torch.empty(sk * m * 2 * n, dtype=torch.float32, device=dev) if mode == 6 else e
                            args = (y, x, wt, mode | tb, wr, kc, sk, True, e, slab, cnt if mode == 6 else e, ssp, 1e-5)
                        try:
                            kern.gemm_decode(*args)
                            torch.cuda.synchronize()
                        except RuntimeError as ex:
                            print(json.dumps({"shape": sname, "proj": proj, "mode": mode, "tile": [wr, kc, sk],
                                              "error": str(ex)[:80]}), flush=True)
                            continue
                        ts = []
                        for _ in range(10):
                            flush.fill_(1)
                            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            t0.record()
                            kern.gemm_decode(*args)
                            t1.record()
                            torch.cuda.synchronize()
                            ts.append(t0.elapsed_time(t1) * 1e3)
                        ts.sort()
                        us = ts[len(ts) // 2]
                        wbytes = w.numel() * 2
                        rec = {"shape": sname, "proj": proj, "N": n, "K": k, "mode": mode, "tile": [wr, kc, sk],
                               "tiled": tiled, "grid": ntiles * sk, "us": round(us, 2),
                               "TBps": round(wbytes / us / 1e6, 2)}
                        print(json.dumps(rec), flush=True)
                        if best is None or us < best["us"]:
                            best = rec
            print(json.dumps({"best": best}), flush=True)


if __name__ == "__main__":
    main()
