"""SiLU-mul microbenchmark at the prefill shape of Llama-3-8B (16,384 tokens x [gate | up] of 14,336)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402


def main():
    t, inter = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (16384, 14336)
    x = torch.randn(t, 2 * inter, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(t, inter, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        ops.silu_and_mul(x, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        ops.silu_and_mul(x, out=out)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 20
    print(json.dumps({"bench": "silu_mul", "tokens": t, "inter": inter, "us": round(us, 1),
                      "TBps": round(3 * t * inter * 2 / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
