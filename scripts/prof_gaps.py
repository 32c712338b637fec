"""GPU idle time of a bench's TIMED region from a rocprofv3 kernel trace (the window between the first and last
`spin_kernel` marker, as scripts/prof_window.py): every gap between one dispatch's end and the next one's start,
summed by size class, and the largest gaps with the kernels on both sides (where the host kept the GPU waiting).

    python scripts/prof_gaps.py <kernel_trace.csv> [--top 25] [--min-us 20]"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--top", type=int, default=25)
ap.add_argument("--min-us", type=float, default=20.0)
ap.add_argument("--context", type=int, default=0, help="dispatches listed around each gap >= 500 us")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[key]]
if len(marks) < 2:
    raise SystemExit("need two spin_kernel markers (run with DIE_PROF_MARKERS=1)")
win = rows[marks[0]: marks[-1] + 1]
t0, t1 = int(win[0]["End_Timestamp"]), int(win[-1]["Start_Timestamp"])
gaps = []
end = int(win[0]["End_Timestamp"])
prev = win[0][key]
big = []
for i, r in enumerate(win[1:], 1):
    s = int(r["Start_Timestamp"])
    if s > end:
        gaps.append(((s - end) / 1e3, prev, r[key]))
        if (s - end) >= 500e3:
            big.append(i)
    if int(r["End_Timestamp"]) > end:
        end, prev = int(r["End_Timestamp"]), r[key]
total = sum(g[0] for g in gaps)
print(f"# GPU idle in the timed window ({(t1 - t0) / 1e6:.1f} ms): {total / 1e3:.2f} ms in {len(gaps)} gaps\n")
cls = defaultdict(lambda: [0, 0.0])
for us, _, _ in gaps:
    c = ("< 5 us" if us < 5 else "5-20 us" if us < 20 else "20-100 us" if us < 100 else "100 us-1 ms" if us < 1000
         else ">= 1 ms")
    cls[c][0] += 1
    cls[c][1] += us
print("| gap size | count | total ms |\n|---|---:|---:|")
for c in ("< 5 us", "5-20 us", "20-100 us", "100 us-1 ms", ">= 1 ms"):
    if c in cls:
        print(f"| {c} | {cls[c][0]} | {cls[c][1] / 1e3:.2f} |")
pairs = defaultdict(lambda: [0, 0.0])
for us, p, n in gaps:
    if us >= a.min_us:
        k = (p[:60], n[:60])
        pairs[k][0] += 1
        pairs[k][1] += us
print(f"\nGaps >= {a.min_us:g} us by (kernel before, kernel after):\n")
print("| count | total ms | before | after |\n|---:|---:|---|---|")
for (p, n), (c, us) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[: a.top]:
    print(f"| {c} | {us / 1e3:.2f} | `{p}` | `{n}` |")
if a.context:
    print(f"\nDispatches around each gap >= 500 us (start relative to the window, duration, queue id):\n")
    for i in big:
        print("```")
        for j in range(max(0, i - a.context), min(len(win), i + a.context)):
            r = win[j]
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            mark = ">>" if j == i else "  "
            print(f"{mark} {(st - t0) / 1e3:10.1f} us {(en - st) / 1e3:8.1f} us q{r.get('Queue_Id', '?')} {r[key][:70]}")
        print("```")
