"""Microbenchmark: cost of a MIXED decode+prefill step's projections — hipBLASLt at M = 32 + chunk
rows against the decode kernel at M = 32 (cold weights: 8 distinct layer copies cycled inside one
hipGraph). Answers: how much does piggybacking a prefill chunk on a decode step add to the step's
weight-streaming projections? One JSON line per (shape, M, variant)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from src import ops  # noqa: E402
from micro_gemm_decode import timeit  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    dev = "cuda:0"
    for name, (n, k) in SHAPES.items():
        ws = [torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(8)]
        for m in (32, 64, 96, 160, 288):
            x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
            us = timeit(lambda w: torch.nn.functional.linear(x, w), ws, iters=32)
            print(json.dumps({"bench": "mixed_gemm", "shape": name, "M": m, "variant": "hipblaslt",
                              "us": round(us, 2), "tb_s": round(n * k * 2 / us / 1e6, 2)}), flush=True)
        x = torch.randn(32, k, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda w: ops.linear(x, w), ws, iters=32)
        print(json.dumps({"bench": "mixed_gemm", "shape": name, "M": 32, "variant": "decode_kernel",
                          "us": round(us, 2), "tb_s": round(n * k * 2 / us / 1e6, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
