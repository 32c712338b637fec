"""Tiny driver for PMC collection: the Llama-3-8B gate/up decode GEMM (cold weights), 40 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn(32, 4096, device=dev, dtype=torch.bfloat16)
ws = [torch.randn(28672, 4096, device=dev, dtype=torch.bfloat16) / 64 for _ in range(8)]
for i in range(40):
    ops.gemm_decode(x, ws[i % 8], 1, 112, 1)
torch.cuda.synchronize()
print("done")
