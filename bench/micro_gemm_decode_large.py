"""Microbenchmark: the decode GEMM at M = 32 / 64 / 128 rows for the Llama-3-8B
projections in the modes the fused decode layer uses (qkv: split-K slabs; o / down: split-K +
last-arriver residual update; gate/up: row-norm scale + SiLU*mul), every (wr, kc, sk) tile that
exists for the row count, tile-order packed weights, against hipBLASLt.

Cold-cache protocol as bench/micro_gemm_decode.py (>= 1.5 GiB of distinct weight copies cycled in a
hipGraph). One JSON line per (shape, M, variant): us per call and effective weight GB/s.

    python bench/micro_gemm_decode_large.py [M ...]
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from micro_gemm_decode import timeit  # noqa: E402

SHAPES = {  # name: (N_out, K, mode)
    "qkv_8b": (6144, 4096, 2),
    "o_8b": (4096, 4096, 3),
    "gate_up_8b": (14336, 4096, 4),
    "down_8b": (4096, 14336, 3),
}
TILES = [(32, 256), (48, 256), (64, 256), (32, 128), (48, 128), (64, 128), (96, 128), (112, 128), (128, 128),
         (64, 64), (128, 64), (64, 32), (128, 32)]


def splits(n, k, mode, wr, kc):
    cols = wr // 2 if mode == 4 else wr
    if n % cols:
        return []
    if mode == 4:
        return [1]
    out = []
    for sk in (1, 2, 4, 8):
        if k % (kc * sk) == 0 and (mode != 3 or wr in (32, 64, 128)):
            t = n // cols * sk
            if 96 <= t <= 1024:
                out.append(sk)
    return out


def main():
    ms = [int(a) for a in sys.argv[1:]] or [32, 64, 128]
    dev = torch.device("cuda:0")
    for name, (n, k, mode) in SHAPES.items():
        rows = 2 * n if mode == 4 else n
        wbytes = rows * k * 2
        copies = max(2, int(1.5 * 2**30 // wbytes) + 1)
        ws = [torch.randn(rows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        for m in ms:
            x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
            res = []
            if mode == 4:
                res.append(("hipblaslt+silu", timeit(lambda w: ops.silu_and_mul(torch.nn.functional.linear(x, w)), ws)))
            else:
                res.append(("hipblaslt", timeit(lambda w: torch.nn.functional.linear(x, w), ws)))
            resid = torch.randn(m, n, device=dev, dtype=torch.bfloat16)
            ssp_in = torch.ones(1, ops.SSP_LD, device=dev) * k
            for wr, kc in TILES:
                for sk in splits(n, k, mode, wr, kc):
                    wts = [ops.gd_pack_weights(w, wr, silu=mode == 4, kc=kc) for w in ws[:2]]
                    wts = (wts * ((copies + 1) // 2))[:copies]
                    try:
                        if mode == 2:
                            fn = lambda w: ops.gemm_decode(x, w, 2 | 32, wr, sk, kc=kc)  # noqa: E731
                        elif mode == 3:
                            ssp = torch.zeros(n // wr, ops.SSP_LD, device=dev)
                            cnt = torch.zeros(n // wr, dtype=torch.int32, device=dev)
                            fn = lambda w, ssp=ssp, cnt=cnt: ops.linear_slab_residual(  # noqa: E731
                                x, w, resid, ssp, cnt, wr, sk, tiled=True, kc=kc)
                        else:
                            fn = lambda w: ops.linear_silu_mul_rownorm(x, w, ssp_in, 1e-5, wr, tiled=True, kc=kc)  # noqa: E731
                        fn(wts[0])
                        torch.cuda.synchronize()
                    except RuntimeError:
                        continue  # no image of this many rows for the tile
                    # the packed copies alias 2 buffers: use real distinct copies for the cold protocol
                    wts = [ops.gd_pack_weights(w, wr, silu=mode == 4, kc=kc) for w in ws]
                    res.append((f"gd_wr{wr}_kc{kc}_sk{sk}", timeit(fn, wts)))
                    del wts
            base = res[0][1]
            for nm, us in sorted(res, key=lambda r: r[1]):
                print(json.dumps({"shape": name, "m": m, "variant": nm, "us": round(us, 2),
                                  "gbps": round(wbytes / us / 1e3, 1), "vs_hipblaslt": round(base / us, 3)}),
                      flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
