"""Decode step tail of Llama-3-8B at 32 rows: final RMSNorm + LM head (128,256 x 4,096, tile-order weights) +
greedy argmax, (a) as the norm kernel, the plain tiled GEMM and the split argmax over the logits (ops.sample with
its scratch), (b) the norm kernel, the GEMM that also writes each column tile's greedy candidate
(ops.linear_tiled_argmax) and the candidate reduction (ops.sample(lm_part=...)). Each form captured 20 times back
to back in one hipGraph, replayed with event timing; random bf16 operands. One JSON line per form, plus the token
agreement of the two. (A third form — the norm as a row scale inside the GEMM from the last down projection's
statistics, no norm kernel — measured 175.7 vs 175.6 us for (b): the per-workgroup statistics load and reduction
in 1,002 LM-head workgroups cost what the norm launch saved; profiles/r5_lm_head_argmax_micro.jsonl. Removed.)

python bench/micro_lm_head_argmax.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    m, n, k, wr, kc, reps = 32, 128256, 4096, 128, 128, 20
    torch.manual_seed(0)
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = ops.gd_pack_weights((torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16), wr, kc=kc)
    samp = (torch.zeros(m * 32, dtype=torch.int32, device=dev), torch.zeros(m, dtype=torch.int32, device=dev))
    parts = torch.zeros(m, n // wr, 2, dtype=torch.int32, device=dev)
    out_a = torch.zeros(m, dtype=torch.long, device=dev)
    out_b = torch.zeros(m, dtype=torch.long, device=dev)
    ones = torch.ones(k, dtype=torch.bfloat16, device=dev)

    def form_a():
        ops.sample(ops.linear_tiled(ops.rms_norm(x, ones, 1e-5), w, wr, kc), out=out_a, scratch=samp)

    def form_b():
        ops.sample(ops.linear_tiled_argmax(ops.rms_norm(x, ones, 1e-5), w, wr, kc, parts), out=out_b, scratch=samp,
                   lm_part=parts)

    res = {}
    for name, fn in (("norm_lm_head_split_argmax", form_a), ("norm_lm_head_candidates", form_b)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / reps)
        ts.sort()
        res[name] = ts[len(ts) // 2]
        print(json.dumps({"bench": "lm_head_argmax", "form": name, "rows": m, "vocab": n, "us_per_step": round(res[name], 2)}),
              flush=True)
    print(json.dumps({"same_tokens": bool(torch.equal(out_a, out_b)),
                      "saved_us": round(res["norm_lm_head_split_argmax"] - res["norm_lm_head_candidates"], 2)}),
          flush=True)


if __name__ == "__main__":
    main()
