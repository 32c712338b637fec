"""Prefill GEMM microbenchmark: y = x @ W^T at M = 16384 tokens (32 x 512 prompts) for the
Llama-3-8B projections on hipBLASLt (the library default the engine's prefill uses).
python bench/micro_prefill_gemm.py [M]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(m, tuned=False):
    dev = torch.device("cuda:0")
    for name, (n, k) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                         "down": (4096, 14336)}.items():
        xs = [torch.randn(m, k, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        ws = [torch.randn(n, k, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        for i in range(3):
            torch.nn.functional.linear(xs[i % 2], ws[i % 2])
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 10
        s.record()
        for i in range(iters):
            torch.nn.functional.linear(xs[i % 2], ws[i % 2])
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        print(json.dumps({"gemm": name, "M": m, "N": n, "K": k, "tuned": tuned, "ms": round(ms, 4),
                          "TFLOPs": round(2 * m * n * k / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    bench(m)
