"""Diagnostic: per-workgroup timeline of the decode GEMM (start / end stamps, s_memrealtime at
100 MHz, and the XCD each workgroup ran on) for the Llama-3-8B decode projections at M = 32,
cold weights. Separates launch-to-first-start, start skew, per-workgroup stream time and the
end-of-kernel straggler tail, i.e. where a projection loses against the chip's stream rate.
Prints one JSON line per shape."""

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src import ops  # noqa: E402

SHAPES = {  # name: (rows of W, N_out, K, mode, wr, sk)
    "qkv": (6144, 6144, 4096, 2, 48, 2),
    "o": (4096, 4096, 4096, 2, 64, 4),
    "gate_up": (28672, 14336, 4096, 1, 112, 1),
    "down": (4096, 4096, 14336, 2, 64, 4),
}


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    tiled = len(sys.argv) > 2 and sys.argv[2] == "tiled"
    dev = torch.device("cuda:0")
    k_ = ops._kern()
    for name, (rows, n, k, mode, wr, sk) in SHAPES.items():
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        copies = max(2, int(1.5 * 2**30 // (rows * k * 2)) + 1)
        ws = [torch.randn(rows, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(copies)]
        ref = ops.gemm_decode(x, ws[0], mode=mode, wr=wr, sk=sk)
        if tiled:  # pre-packed tile-order weights (ops.gd_pack_weights): same math, linear DMA pieces
            ws = [ops.gd_pack_weights(w_, wr, silu=mode == 1) for w_ in ws]
            mode |= 32
            got = ops.gemm_decode(x, ws[0], mode=mode, wr=wr, sk=sk)
            assert torch.equal(got, ref), (name, (got.float() - ref.float()).abs().max())
        cols = wr // 2 if (mode & 31) == 1 else wr
        nwg = (n // cols) * sk
        ts = torch.zeros(copies, 3 * nwg, dtype=torch.int64, device=dev)
        outs = []
        for i in range(copies):
            ops.gemm_decode(x, ws[i], mode=mode, wr=wr, sk=sk)   # warm the code / allocator
        torch.cuda.synchronize()
        for i in range(copies):
            k_.gd_set_timestamps(ts[i])
            outs.append(ops.gemm_decode(x, ws[i], mode=mode, wr=wr, sk=sk))
        k_.gd_set_timestamps(torch.empty(0, dtype=torch.int64, device=dev))
        torch.cuda.synchronize()
        t = ts.view(copies, nwg, 3).cpu()
        spans, skews, tails, durs_med, durs_max = [], [], [], [], []
        xcd_end = {}
        for i in range(2, copies):   # skip the first launches
            st, en, xc = t[i, :, 0].double(), t[i, :, 1].double(), t[i, :, 2]
            t0 = st.min()
            spans.append(float(en.max() - t0) * 10e-3)
            skews.append(float(st.max() - t0) * 10e-3)
            tails.append(float(en.max() - en.median()) * 10e-3)
            d = (en - st) * 10e-3
            durs_med.append(float(d.median()))
            durs_max.append(float(d.max()))
            for x_ in range(8):
                sel = xc == x_
                if sel.any():
                    xcd_end.setdefault(x_, []).append(float(en[sel].max() - t0) * 10e-3)
        wbytes = rows * k * 2
        span = statistics.median(spans)
        print(json.dumps({"shape": name, "m": m, "tiled": tiled, "workgroups": nwg, "span_us": round(span, 2),
                          "start_skew_us": round(statistics.median(skews), 2),
                          "tail_after_median_end_us": round(statistics.median(tails), 2),
                          "wg_dur_median_us": round(statistics.median(durs_med), 2),
                          "wg_dur_max_us": round(statistics.median(durs_max), 2),
                          "tb_per_s_span": round(wbytes / span / 1e6, 2),
                          "xcd_last_end_us": {x_: round(statistics.median(v), 2) for x_, v in sorted(xcd_end.items())}}),
              flush=True)


if __name__ == "__main__":
    main()
