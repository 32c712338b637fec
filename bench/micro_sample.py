"""Greedy sampling of a decode step's logits (32 rows x 128,256 bf16, Llama-3 vocab): one workgroup per row
against the split form (ops.sample with scratch: each row's argmax over up to 16 workgroups, last arriver
combines). Median of 50 event-timed calls; one JSON line per form; the split result is checked against torch.

python bench/micro_sample.py [--rows 32] [--vocab 128256]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--vocab", type=int, default=128256)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    logits = torch.randn(a.rows, a.vocab, device=dev).to(torch.bfloat16)
    scratch = (torch.zeros(a.rows * 32, dtype=torch.int32, device=dev),
               torch.zeros(a.rows, dtype=torch.int32, device=dev))
    want = logits.float().argmax(-1)
    for name, sc in (("one_wg_per_row", None), ("split", scratch)):
        out = ops.sample(logits, scratch=sc)
        torch.cuda.synchronize()
        assert torch.equal(out, want), name
        ts = []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.sample(logits, out=out, scratch=sc)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(json.dumps({"bench": "sample_greedy", "form": name, "rows": a.rows, "vocab": a.vocab,
                          "us": round(ts[len(ts) // 2], 2)}), flush=True)


if __name__ == "__main__":
    main()
