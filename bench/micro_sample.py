"""Greedy sampling (argmax pass) of 32 x 128,256 bf16 logits: microseconds per call (100 back-to-back calls)."""
import json, sys, torch
sys.path.insert(0, ".")
from src import ops
dev = torch.device("cuda:0")
lg = (torch.randn(32, 128256, device=dev) * 3).to(torch.bfloat16)
out = torch.empty(32, dtype=torch.long, device=dev)
for _ in range(5):
    ops.sample(lg, out=out)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(100):
    ops.sample(lg, out=out)
b.record(); torch.cuda.synchronize()
print(json.dumps({"bench": "sample_greedy", "rows": 32, "vocab": 128256, "us_per_call": round(a.elapsed_time(b) * 10, 2)}))
