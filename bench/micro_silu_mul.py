"""SiLU-mul microbenchmark at the prefill shape of Llama-3-8B (16,384 tokens x [gate | up] of 14,336): the
launcher's default decomposition and every chunks-per-lane count, on the [T, 2I] layout and on the two column
halves of [T, I] chunk buffers (the layout of an FFN run in two column chunks, bench/micro_ffn_nchunk.py).

python bench/micro_silu_mul.py [tokens inter]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n


def main():
    t, inter = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (16384, 14336)
    x = torch.randn(t, 2 * inter, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(t, inter, device="cuda", dtype=torch.bfloat16)
    c = inter // 2
    halves = [torch.randn(t, 2 * c, device="cuda", dtype=torch.bfloat16) for _ in range(2)]

    def row(layout, per, us):
        print(json.dumps({"bench": "silu_mul", "layout": layout, "tokens": t, "inter": inter, "per": per,
                          "us": round(us, 1), "TBps": round(3 * t * inter * 2 / us / 1e6, 2)}), flush=True)

    row("default [T,2I]", "auto", timed(lambda: ops.silu_and_mul(x, out=out)))
    for per in range(0, 9):
        row("views [T,2I]", per, timed(lambda: ops.silu_and_mul_views(x[:, :inter], x[:, inter:], out, per=per)))

    def two(per):
        for i, h in enumerate(halves):
            ops.silu_and_mul_views(h[:, :c], h[:, c:], out[:, c * i:c * (i + 1)], per=per)

    for per in range(0, 9):
        row("2 chunks [T,I]", per, timed(lambda: two(per)))
    ref = ops.silu_and_mul(x)
    ops.silu_and_mul_views(x[:, :inter], x[:, inter:], out, per=3)
    print(json.dumps({"check_per3_vs_default": float((ref.float() - out.float()).abs().max())}))


if __name__ == "__main__":
    main()
