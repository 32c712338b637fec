"""Prefill GEMM table for PyTorch TunableOp: every hipBLASLt / rocBLAS solution is timed for each prefill
projection shape (dense Llama-3 8B / 70B shapes, TP = 1 / 2 / 8 shards, token counts of typical prefill
steps) and the fastest kept, vs the library's default heuristic choice. Event-timed medians of 10 calls, random
bf16 operands (DVFS-representative). One JSON line per shape; the table (validators: PyTorch, HIP, hipBLASLt,
rocBLAS versions, gfx950) is written to --out, which ``src.ops.gemm_table`` loads read-only at engine start.

python bench/micro_prefill_tunableop.py --out gpurun_out/tunableop_prefill.csv [--quick]
"""
import argparse
import json

import torch

# (model shard, [(proj, N, K)]) — x [M, K] @ w[N, K]^T as torch.nn.functional.linear runs it
SHAPES = {
    "8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)],
    "8b_tp2": [("qkv", 3072, 4096), ("o", 4096, 2048), ("gate_up", 14336, 4096), ("down", 4096, 7168)],
    "70b_tp8": [("qkv", 1280, 8192), ("o", 8192, 1024), ("gate_up", 7168, 8192), ("down", 8192, 3584)],
    "70b": [("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192), ("down", 8192, 28672)],
}
TOKENS = {"8b": (16384, 8192, 4096, 2048), "8b_tp2": (16384, 8192), "70b_tp8": (16384, 8192), "70b": (16384,)}


def timed(fn, n=10):
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
    ap.add_argument("--out", default="gpurun_out/tunableop_prefill.csv")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--models", default="8b,8b_tp2,70b_tp8,70b")
    ap.add_argument("--quick", action="store_true", help="8B at 16,384 tokens only")
    ap.add_argument("--residual", action="store_true",
                    help="the o / down projections only, as the one-GPU prefill runs them: resid += x @ w^T in place "
                         "(ops.linear_residual, beta = 1)")
    a = ap.parse_args()
    import torch.cuda.tunable as tun

    dev = torch.device("cuda:0")
    todo = []
    for mdl in a.models.split(","):
        for m in (TOKENS[mdl][:1] if a.quick else TOKENS[mdl]):
            for proj, n, k in SHAPES[mdl]:
                if not a.residual or proj in ("o", "down"):
                    todo.append((mdl, proj, m, n, k))
        if a.quick:
            break
    def operands(m, n, k):
        x = torch.randn(m, k, device=dev).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
        r = torch.randn(m, n, device=dev).to(torch.bfloat16) if a.residual else None
        return x, w, r

    def gemm(x, w, r):
        return r.addmm_(x, w.t()) if r is not None else torch.nn.functional.linear(x, w)

    base = {}
    for key in todo:
        _, _, m, n, k = key
        x, w, r = operands(m, n, k)
        gemm(x, w, r)
        torch.cuda.synchronize()
        base[key] = timed(lambda: gemm(x, w, r))
        del x, w, r
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_iterations(a.iters)
    tun.set_filename(a.out)
    for key in todo:
        _, _, m, n, k = key
        x, w, r = operands(m, n, k)
        gemm(x, w, r)  # tunes this shape
        torch.cuda.synchronize()
        print(json.dumps({"tuned": list(key)}), flush=True)  # progress (a long silence reads as a hang)
        del x, w, r
    tun.tuning_enable(False)
    for key in todo:
        mdl, proj, m, n, k = key
        x, w, r = operands(m, n, k)
        t = timed(lambda: gemm(x, w, r))
        fl = 2 * m * n * k
        print(json.dumps({"bench": "prefill_tunableop", "model": mdl, "proj": proj, "M": m, "N": n, "K": k,
                          "residual_beta1": a.residual,
                          "default_us": round(base[key], 1), "tuned_us": round(t, 1),
                          "default_PFs": round(fl / base[key] / 1e9, 3), "tuned_PFs": round(fl / t / 1e9, 3)}),
              flush=True)
        del x, w, r
    if hasattr(tun, "write_file"):  # newer PyTorch writes the file named by set_filename at exit
        tun.write_file(a.out)


if __name__ == "__main__":
    main()
