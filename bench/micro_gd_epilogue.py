"""What the residual-updating epilogue of the decode GEMM costs: the o-proj and down-proj of
Llama-3-8B at M = 32 with the decode plan's tile (64 rows, K slot 256, split-K 4, tile-order weights),
in mode 2 (split-K fp32 slabs only, reduced by the consumer) and mode 3 (slabs + the split-K last
arriver adding into the residual and writing the next norm's row statistics). Cold weights, launches
replayed back to back from a hipGraph (bench/micro_gemm_decode.py timeit).

    python bench/micro_gd_epilogue.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from micro_gemm_decode import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    m = 32
    for name, (n, k) in {"o_8b": (4096, 4096), "down_8b": (4096, 14336)}.items():
        copies = max(2, int(1.5 * 2**30 // (n * k * 2)) + 1)
        ws = [ops.gd_pack_weights(torch.randn(n, k, device=dev, dtype=torch.bfloat16) / 64, 64, kc=256)
              for _ in range(copies)]
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        resid = torch.randn(m, n, device=dev, dtype=torch.bfloat16)
        ssp = torch.zeros(n // 64, ops.SSP_LD, device=dev)
        cnt = torch.zeros(n // 64, dtype=torch.int32, device=dev)
        slab = torch.empty(4, m, n, device=dev)
        res = {"shape": name, "m": m}
        for sk in (1, 2, 4):
            if k % (256 * sk):
                continue
            sl = torch.empty(sk, m, n, device=dev)
            res[f"mode2_sk{sk}_us"] = round(timeit(lambda w, sl=sl, sk=sk: ops.gemm_decode(x, w, 2 | 32, 64, sk, out=sl, kc=256), ws), 2)
            res[f"mode3_sk{sk}_us"] = round(timeit(lambda w, sk=sk: ops.linear_slab_residual(x, w, resid, ssp, cnt, 64, sk, tiled=True, kc=256), ws), 2)
        print(json.dumps(res), flush=True)
        del ws, slab


if __name__ == "__main__":
    main()
