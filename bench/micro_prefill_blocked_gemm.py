"""Can prefill's hipBLASLt GEMMs run on a column-blocked weight layout as fast as on the row-major one?

Layout [N / WR][K][WR]: each block of WR output columns is a row-major [K, WR] matrix (W^T of the block), i.e.
every (WR x KC) chunk a decode-GEMM workgroup streams is contiguous. Prefill then runs ONE strided-batched GEMM
(batch = N / WR, A = the activations with batch stride 0, C = the [M, N] output viewed as [N / WR, M, WR] with
ldc = N, batch stride WR). Times each Llama-3-8B projection at the bench's 16,384-row wave against F.linear on
the row-major weight; also checks that the result is identical. One JSON line per (projection, WR)."""

import json
import sys

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    for name, (n, k) in SHAPES.items():
        x = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(n, k, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
        y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        base = timeit(lambda: F.linear(x, w, out=y))
        ref = y.clone()
        flops = 2.0 * m * n * k
        for wr in (64, 128, 256):
            nb = n // wr
            wb = w.view(nb, wr, k).transpose(1, 2).contiguous()       # [nb, K, WR]
            yb = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
            out = yb.view(m, nb, wr).transpose(0, 1)                    # [nb, M, WR], strides (WR, N, 1)
            xa = x.unsqueeze(0).expand(nb, m, k)
            ok = True
            try:
                torch.bmm(xa, wb, out=out)
            except RuntimeError as e:
                ok = str(e)[:120]
            t = timeit(lambda: torch.bmm(xa, wb, out=out)) if ok is True else None
            same = bool(torch.equal(yb, ref)) if ok is True else None
            print(json.dumps({"bench": "prefill_blocked_gemm", "proj": name, "M": m, "N": n, "K": k, "WR": wr,
                              "row_major_us": round(base, 1), "blocked_us": round(t, 1) if t else None,
                              "row_major_PFs": round(flops / base / 1e9, 3),
                              "blocked_PFs": round(flops / t / 1e9, 3) if t else None,
                              "ratio": round(base / t, 3) if t else None, "identical": same, "error": ok}),
                  flush=True)


if __name__ == "__main__":
    main()
