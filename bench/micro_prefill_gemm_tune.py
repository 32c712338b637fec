"""Prefill-step GEMMs at small M (one or a few prompts: M = 512 / 1024 / 2048 tokens) — hipBLASLt's
default choice vs PyTorch TunableOp tuned on this GPU (hipBLASLt + rocBLAS solutions timed online).
Llama-3-8B projection shapes. Prints us per GEMM and the winning solution names.

    python bench/micro_prefill_gemm_tune.py [out.csv]
"""
import json
import os
import sys

import torch

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
MS = (512, 1024, 2048)


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_small_m.csv"
    dev = torch.device("cuda:0")
    ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) / 64 for k, (n, kk) in SHAPES.items()}
    xs = {(m, kk): torch.randn(m, kk, device=dev, dtype=torch.bfloat16) for m in MS for kk in (4096, 14336)}
    base = {}
    for name, (n, k) in SHAPES.items():
        for m in MS:
            base[(name, m)] = timeit(lambda: torch.nn.functional.linear(xs[(m, k)], ws[name]))
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(out, insert_device_ordinal=False)
    tun.set_max_tuning_duration(30)
    tun.set_max_tuning_iterations(20)
    for name, (n, k) in SHAPES.items():
        for m in MS:
            torch.nn.functional.linear(xs[(m, k)], ws[name])  # tunes this shape
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    for name, (n, k) in SHAPES.items():
        for m in MS:
            us = timeit(lambda: torch.nn.functional.linear(xs[(m, k)], ws[name]))
            fl = 2 * m * n * k
            print(json.dumps({"bench": "prefill_gemm_tune", "shape": name, "m": m, "default_us": round(base[(name, m)], 1),
                              "tuned_us": round(us, 1), "default_pfs": round(fl / base[(name, m)] / 1e9, 3),
                              "tuned_pfs": round(fl / us / 1e9, 3)}), flush=True)
    if hasattr(tun, "write_file_on_exit"):
        tun.write_file_on_exit(True)


if __name__ == "__main__":
    main()
