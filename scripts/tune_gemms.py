"""Tune the prefill GEMM shapes with PyTorch TunableOp (hipBLASLt + rocBLAS solutions,
timed on this GPU) and write the winners to configs/tunableop_results0.csv, which the engine
loads at start-up (src/ops/gemm_tuning.py) with tuning itself disabled.

python scripts/tune_gemms.py [out.csv]
"""
import os
import sys
import time

import torch

out = sys.argv[1] if len(sys.argv) > 1 else "configs/tunableop_results0.csv"
os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(out, insert_device_ordinal=False)
tun.set_max_tuning_duration(60)
tun.set_max_tuning_iterations(30)
dev = torch.device("cuda:0")
SHAPES = [  # (N, K): Llama-3-8B / Mixtral attention, Llama-3-8B MLP, Llama-3-70B TP=8 shards
    (6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336),
    (1280, 8192), (8192, 1024), (7168, 8192), (8192, 3584),
]
MS = [16384, 8192, 4096, 2048, 1024, 512]
t0 = time.time()
for n, k in SHAPES:
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    for m in MS:
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        t1 = time.time()
        torch.nn.functional.linear(x, w)
        torch.cuda.synchronize()
        print(f"tuned M={m} N={n} K={k} in {time.time() - t1:.1f}s (total {time.time() - t0:.0f}s)", flush=True)
tun.write_file()
print("wrote", out, flush=True)
