"""The decode GEMM's split-K SiLU form (mode 6: K split over sk workgroups per tile, fp32 partial slabs, the
tile's last arriver applies the norm row scale and SiLU*mul) against the single-pass mode 4, for gate/up
projections where the full-K form needs narrow tiles to fill the grid: Llama-3-70B's TP=8 shard (3,584
outputs, K 8,192) and Llama-3-8B (14,336 outputs, K 4,096) at 32 / 64 / 128 rows. Tile-order weights, cold
(a 1 GiB buffer written before every call), median of 10 event-timed calls. One JSON line per variant.

python bench/micro_gd_splitk_silu.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    kern = ops._kern()
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    e = torch.empty(0, device=dev)
    cases = [("gate_up_70b_tp8", 3584, 8192, (32,)), ("gate_up_8b", 14336, 4096, (32, 64, 128))]
    tiles4 = [(32, 256), (64, 256), (64, 128), (112, 128), (128, 128), (128, 64), (64, 64)]
    tiles6 = [(64, 256, 2), (64, 128, 2), (112, 128, 2), (128, 128, 2), (128, 128, 4), (128, 64, 2), (128, 64, 4),
              (112, 128, 4), (64, 128, 4)]
    for name, n, k, rows in cases:
        w = (torch.randn(2 * n, k, device=dev) * 0.02).to(torch.bfloat16)
        ssp = (torch.rand(4, 128, device=dev) * k * 0.1).float()
        for m in rows:
            x = torch.randn(m, k, device=dev).to(torch.bfloat16)
            ref = None
            for wr, kc, sk, mode in [(a, b, 1, 4) for a, b in tiles4] + [(a, b, c, 6) for a, b, c in tiles6]:
                if n % (wr // 2) or k % (kc * sk) or not ops.gd_tile_valid(wr, kc, max(16, m if m > 16 else 32)):
                    continue
                wt = ops.gd_pack_weights(w, wr, silu=True, kc=kc)
                y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
                slab = torch.empty(sk * m * 2 * n, dtype=torch.float32, device=dev) if mode == 6 else e
                cnt = torch.zeros(n // (wr // 2), dtype=torch.int32, device=dev)

                def run():
                    kern.gemm_decode(y, x, wt, mode | 32, wr, kc, sk, True, e, slab if mode == 6 else e,
                                     cnt if mode == 6 else e, ssp, 1e-5)
                try:
                    run()
                except RuntimeError as ex:
                    print(json.dumps({"shape": name, "rows": m, "mode": mode, "tile": [wr, kc, sk],
                                      "error": str(ex)[:100]}), flush=True)
                    continue
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.float().clone()
                err = float((y.float() - ref).norm() / ref.norm())
                ts = []
                for _ in range(10):
                    flush.fill_(1)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    run()
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b) * 1e3)
                ts.sort()
                us = ts[len(ts) // 2]
                print(json.dumps({"shape": name, "rows": m, "mode": mode, "tile": [wr, kc, sk], "us": round(us, 2),
                                  "TBps": round(2 * n * k * 2 / us / 1e6, 2), "rel_err_vs_first": round(err, 6),
                                  "counters_rearmed": int(cnt.abs().sum())}), flush=True)


if __name__ == "__main__":
    main()
