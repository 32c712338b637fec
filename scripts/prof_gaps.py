"""Idle-time anatomy of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

    python scripts/prof_gaps.py <..._kernel_trace.csv> [decode-marker-substring]

Sorts dispatches by start time and splits the GPU-idle time between consecutive kernels into
buckets (< 5 us: in-graph dispatch gaps; 5-50 us: between graph replays; 50 us - 2 ms: host
round trips; > 2 ms: phase changes / warmup). With a marker (default: the decode attention
kernel), it also reports, for the decode region only (first to last marker dispatch), the
busy/idle split per decode step (steps counted by the LM-head dispatches, the gemm_decode
kernel with mode 0)."""

import csv
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "attn_decode_v3"
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    idx = [i for i, k in enumerate(ks) if marker in k[2]]
    if not idx:
        print("marker not found")
        return
    lo, hi = idx[0], idx[-1]
    # extend to the whole decode step around the markers: include the LM head / sampling of the last step
    while hi + 1 < len(ks) and ("gemm_decode" in ks[hi + 1][2] or "sample" in ks[hi + 1][2]
                                or "decode_advance" in ks[hi + 1][2] or "rmsnorm" in ks[hi + 1][2]):
        hi += 1
    seg = ks[lo: hi + 1]
    busy = sum(e - s for s, e, _ in seg)
    span = seg[-1][1] - seg[0][0]
    buckets = Counter()
    bucket_n = Counter()
    end = seg[0][1]
    for s, e, _ in seg[1:]:
        gap = max(0, s - end)
        b = "<5us" if gap < 5e3 else "5-50us" if gap < 5e4 else "50us-2ms" if gap < 2e6 else ">2ms"
        buckets[b] += gap
        bucket_n[b] += 1
        end = max(end, e)
    steps = sum(1 for _, _, n in seg if "gemm_decode_kernel<64, 0" in n) or 1
    print(f"decode region: {len(seg)} dispatches, {steps} steps, span {span/1e6:.2f} ms, busy {busy/1e6:.2f} ms "
          f"({100*busy/span:.1f} %)")
    print(f"per step: span {span/steps/1e3:.1f} us, busy {busy/steps/1e3:.1f} us, idle {(span-busy)/steps/1e3:.1f} us")
    for b in ("<5us", "5-50us", "50us-2ms", ">2ms"):
        print(f"  gaps {b:>9}: {bucket_n[b]:6d} x, total {buckets[b]/1e6:8.3f} ms, per step {buckets[b]/steps/1e3:7.1f} us")


if __name__ == "__main__":
    main()
