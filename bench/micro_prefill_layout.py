"""Prefill GEMM operand layout: y[M, N] = x[M, K] @ W^T with the weight stored row-major [N, K] (what the model
keeps: torch.nn.functional.linear) vs stored transposed [K, N] (torch.matmul(x, Wt)), for the Llama-3-8B
projections at 16,384 tokens. Both layouts timed with the library's default solution and after PyTorch TunableOp
tuned each shape (every hipBLASLt / rocBLAS solution). Event-timed medians, random bf16 operands.

python bench/micro_prefill_layout.py
"""
import json

import torch

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]


def timed(fn, n=12):
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
    import torch.cuda.tunable as tun

    dev = torch.device("cuda:0")
    m = 16384
    ops = {}
    for name, n, k in SHAPES:
        x = torch.randn(m, k, device=dev).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
        wt = w.t().contiguous()
        ops[name] = (lambda x=x, w=w: torch.nn.functional.linear(x, w),
                     lambda x=x, wt=wt: torch.matmul(x, wt), 2 * m * n * k)
    res = {}
    for name, (f_nk, f_kn, fl) in ops.items():
        f_nk(), f_kn()
        torch.cuda.synchronize()
        res[name] = [timed(f_nk), timed(f_kn)]
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_iterations(20)
    tun.set_filename("/tmp/prefill_layout_tune.csv")
    for name, (f_nk, f_kn, fl) in ops.items():
        f_nk(), f_kn()
        torch.cuda.synchronize()
        print(json.dumps({"tuned": name}), flush=True)
    tun.tuning_enable(False)
    for name, (f_nk, f_kn, fl) in ops.items():
        f_nk(), f_kn()
        torch.cuda.synchronize()
        t_nk, t_kn = timed(f_nk), timed(f_kn)
        d_nk, d_kn = res[name]
        print(json.dumps({"bench": "prefill_layout", "proj": name, "M": m, "flop": fl,
                          "default_us": {"w[N,K]": round(d_nk, 1), "w[K,N]": round(d_kn, 1)},
                          "tuned_us": {"w[N,K]": round(t_nk, 1), "w[K,N]": round(t_kn, 1)},
                          "tuned_PFs": {"w[N,K]": round(fl / t_nk / 1e9, 3), "w[K,N]": round(fl / t_kn / 1e9, 3)}}),
              flush=True)


if __name__ == "__main__":
    main()
