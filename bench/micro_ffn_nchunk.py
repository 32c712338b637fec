"""Prefill FFN front half in column chunks: gate/up GEMM + SiLU·up for 16,384 tokens of Llama-3-8B, done
(a) in one GEMM [M, 28,672] followed by one SiLU·up pass, or (b) in chunks of c intermediate columns: a
GEMM [M, 2c] on the chunk's gate and up weight rows, then SiLU·up of that chunk while its GEMM output is
still in the Infinity Cache (2c columns x 16,384 rows x 2 B: 64 MiB at c = 1,024, 224 MiB at c = 3,584).

Event-timed medians of --iters calls, random bf16 operands; optional PyTorch TunableOp for the chunk
shapes (--tune: every hipBLASLt / rocBLAS solution timed, the fastest used for both arms).
One JSON line per arm.

Result (profiles/r5_ffn_nchunk_micro.jsonl): two column blocks on a chunk-interleaved weight copy ran the pair
1.6-2.7 % faster than one GEMM + one pass here (the SiLU * up pass after each block 230-250 us vs 260-335), but
the same layout in the served model (CausalLM.pack_ffn_blocks, built and removed) did not move the bench's prefill
(0.483 / 0.485 s vs 0.484 / 0.486 s per 3 waves, profiles/r5_ffn_blocks_bench_ab_negative.jsonl).

python bench/micro_ffn_nchunk.py [--tune]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n):
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--chunks", default="1024,2048,3584,7168")
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--mrows", default="8192,4096")
    ap.add_argument("--tune", action="store_true")
    a = ap.parse_args()
    from src import ops  # noqa: E402

    dev = torch.device("cuda:0")
    m, k, inter = a.tokens, a.hidden, a.inter
    torch.manual_seed(0)
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(2 * inter, k, device=dev) * 0.02).to(torch.bfloat16)  # [gate; up]
    rs = torch.rand(m, device=dev) + 0.5
    act = torch.empty(m, inter, device=dev, dtype=torch.bfloat16)
    chunks = [int(c) for c in a.chunks.split(",")]
    if a.tune:
        import torch.cuda.tunable as tun

        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_iterations(20)
        tun.set_filename("/tmp/ffn_nchunk_tune.csv")
    # chunk-interleaved copies of the weights: rows [gate c-block i; up c-block i] contiguous per chunk
    perm = {}
    for c in chunks:
        idx = torch.arange(2 * inter, device=dev).view(2, inter // c, c).transpose(0, 1).reshape(-1)
        perm[c] = w.index_select(0, idx)
    y_full = torch.empty(m, 2 * inter, device=dev, dtype=torch.bfloat16)

    def full():
        torch.matmul(x, w.t(), out=y_full)
        ops.silu_and_mul(y_full, act, rs)

    def gemm_only():
        torch.matmul(x, w.t(), out=y_full)

    bufs = {c: torch.empty(m, 2 * c, device=dev, dtype=torch.bfloat16) for c in chunks}
    outs = {c: torch.empty(m, c, device=dev, dtype=torch.bfloat16) for c in chunks}

    def chunked(c, silu=True):
        wp, yb, ob = perm[c], bufs[c], outs[c]
        for i in range(inter // c):
            torch.matmul(x, wp[2 * c * i:2 * c * (i + 1)].t(), out=yb)
            if silu:
                ops.silu_and_mul(yb, ob, rs)

    # (c) no weight permutation: per chunk, one GEMM on the gate rows and one on the up rows of the
    # row-major [gate; up] weight, SiLU * up of the two column views into the activation's columns
    def split(c, silu=True):
        yb = bufs[c]
        for i in range(inter // c):
            torch.matmul(x, w[c * i:c * (i + 1)].t(), out=yb[:, :c])
            torch.matmul(x, w[inter + c * i:inter + c * (i + 1)].t(), out=yb[:, c:])
            if silu:
                ops.silu_and_mul_views(yb[:, :c], yb[:, c:], act[:, c * i:c * (i + 1)], rs)

    # (d) row chunks: the whole [gate; up] weight on r rows of tokens at a time, SiLU * up per row block
    mrows = [int(r) for r in a.mrows.split(",")]
    ybm = {r: torch.empty(r, 2 * inter, device=dev, dtype=torch.bfloat16) for r in mrows}

    def mchunk(r, silu=True):
        yb = ybm[r]
        for i in range(m // r):
            torch.matmul(x[r * i:r * (i + 1)], w.t(), out=yb)
            if silu:
                ops.silu_and_mul(yb, act[r * i:r * (i + 1)], rs[r * i:r * (i + 1)])

    # warm-up (and tuning, when enabled) of every shape
    def warm():
        full()
        for c in chunks:
            chunked(c)
            split(c)
        for r in mrows:
            mchunk(r)
        torch.cuda.synchronize()

    warm()
    if a.tune:
        tun.tuning_enable(False)
        warm()
    fl = 2 * m * 2 * inter * k
    t_full, t_g = timed(full, a.iters), timed(gemm_only, a.iters)
    print(json.dumps({"bench": "ffn_nchunk", "chunk": inter, "tune": a.tune, "total_us": round(t_full, 1),
                      "gemm_us": round(t_g, 1), "silu_us": round(t_full - t_g, 1),
                      "gemm_PFs": round(fl / t_g / 1e9, 3)}), flush=True)
    for c in chunks:
        t, tg = timed(lambda: chunked(c), a.iters), timed(lambda: chunked(c, False), a.iters)
        print(json.dumps({"bench": "ffn_nchunk", "chunk": c, "tune": a.tune, "total_us": round(t, 1),
                          "gemm_us": round(tg, 1), "silu_us": round(t - tg, 1),
                          "gemm_PFs": round(fl / tg / 1e9, 3), "vs_full": round(t / t_full, 4)}), flush=True)
    for c in chunks:
        t, tg = timed(lambda: split(c), a.iters), timed(lambda: split(c, False), a.iters)
        print(json.dumps({"bench": "ffn_nchunk_split", "chunk": c, "tune": a.tune, "total_us": round(t, 1),
                          "gemm_us": round(tg, 1), "silu_us": round(t - tg, 1),
                          "gemm_PFs": round(fl / tg / 1e9, 3), "vs_full": round(t / t_full, 4)}), flush=True)
    for r in mrows:
        t, tg = timed(lambda: mchunk(r), a.iters), timed(lambda: mchunk(r, False), a.iters)
        print(json.dumps({"bench": "ffn_mchunk", "rows": r, "tune": a.tune, "total_us": round(t, 1),
                          "gemm_us": round(tg, 1), "silu_us": round(t - tg, 1),
                          "gemm_PFs": round(fl / tg / 1e9, 3), "vs_full": round(t / t_full, 4)}), flush=True)
    ref_act = act.clone()
    full()
    torch.cuda.synchronize()
    print(json.dumps({"check_split_or_rows_vs_full": float((ref_act.float() - act.float()).abs().max())}), flush=True)
    # numerics: the chunked form equals the full form column block by column block
    full()
    c = chunks[0]
    wp, yb, ob = perm[c], bufs[c], outs[c]
    torch.matmul(x, wp[:2 * c].t(), out=yb)
    ops.silu_and_mul(yb, ob, rs)
    torch.cuda.synchronize()
    print(json.dumps({"check_max_abs_diff": float((ob.float() - act[:, :c].float()).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
