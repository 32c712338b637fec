"""Microbenchmark: the decode MLP half (Llama-3-8B, M = 32) as two launches (gate/up mode 4 +
down mode 3) vs one persistent launch (ops.mlp_decode), cold weights (8 distinct layer copies,
2.8 GB, cycled inside one captured hipGraph). Prints one JSON line per variant: µs per layer
and effective weight-stream TB/s."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from src import ops  # noqa: E402
from micro_gemm_decode import timeit  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    h, inter, nl = 4096, 14336, 8
    dev = "cuda:0"
    layers = [(torch.randn(2 * inter, h, device=dev, dtype=torch.bfloat16) * 0.02,
               torch.randn(h, inter, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(nl)]
    x = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    ssp = torch.zeros(64, 32, device=dev)
    ssp[:, :m] = x.float().pow(2).view(m, 64, 64).sum(-1).t()
    ssp_out = torch.zeros(64, 32, device=dev)
    cnt = torch.zeros(64, dtype=torch.int32, device=dev)
    flags = torch.zeros(8, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    act = torch.empty(m, inter, dtype=torch.bfloat16, device=dev)
    slab = torch.empty(4 * m * h, dtype=torch.float32, device=dev)
    resid = x.clone()
    nbytes = (3 * inter * h) * 2

    def two(w):
        a = ops.linear_silu_mul_rownorm(x, w[0], ssp, 1e-5, 112)
        ops.linear_slab_residual(a, w[1], resid, ssp_out, cnt, 64, 4)

    def fused(w):
        ops.mlp_decode(x, w[0], w[1], ssp, 1e-5, resid, ssp_out, cnt, flags, err, act, slab)

    def gate_up(w):
        ops.linear_silu_mul_rownorm(x, w[0], ssp, 1e-5, 112)

    def down(w):
        ops.linear_slab_residual(act, w[1], resid, ssp_out, cnt, 64, 4)

    for name, fn, b in (("two_launches", two, nbytes), ("persistent", fused, nbytes),
                        ("gate_up_only", gate_up, 2 * inter * h * 2), ("down_only", down, inter * h * 2)):
        us = timeit(fn, layers, iters=32)
        print(json.dumps({"bench": "mlp_decode", "m": m, "variant": name, "us": round(us, 2),
                          "tb_s": round(b / us / 1e6, 2)}), flush=True)
    assert int(err.item()) == 0


if __name__ == "__main__":
    main()
