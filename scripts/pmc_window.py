"""Per-kernel counter table of a bench's TIMED region from a rocprofv3 `--pmc ... --kernel-trace` CSV run: keeps
the dispatches between the first and the last `spin_kernel` marker (DIE_PROF_MARKERS=1) and reports, per kernel
name, the mean of each counter per call and — for FETCH_SIZE / WRITE_SIZE (KiB) — the bytes per call and the
rate over the kernel-trace duration of the same dispatches.

    python scripts/pmc_window.py <counter_collection.csv> <kernel_trace.csv> [title] [--per STEPS] [--n N]
"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("counters")
ap.add_argument("trace")
ap.add_argument("title", nargs="?", default=None)
ap.add_argument("--per", type=float, default=0.0)
ap.add_argument("--n", type=int, default=14)
a = ap.parse_args()

trace = list(csv.DictReader(open(a.trace)))
key = "Kernel_Name" if "Kernel_Name" in trace[0] else "Name"
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(trace) if "spin_kernel" in r[key]]
if len(marks) < 2:
    raise SystemExit("need two spin_kernel markers (run with DIE_PROF_MARKERS=1)")
win = trace[marks[0] + 1: marks[-1]]
ids = {r["Dispatch_Id"]: r for r in win}

vals = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value (summed over instances)
for r in csv.DictReader(open(a.counters)):
    d = r.get("Dispatch_Id")
    if d in ids:
        vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
counters = sorted({c for v in vals.values() for c in v})

agg = defaultdict(lambda: {"n": 0, "ns": 0, **{c: 0.0 for c in counters}})
for d, r in ids.items():
    g = agg[r[key]]
    g["n"] += 1
    g["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for c in counters:
        g[c] += vals[d].get(c, 0.0)

print(f"# {a.title or a.counters}\n")
print(f"{len(win)} dispatches between the markers; counters: {', '.join(counters)} (per call; KiB for the "
      f"*_SIZE counters, rate = bytes / the dispatch's kernel-trace time)\n")
cols = ["calls", "us/call"] + [f"{c}/call" for c in counters]
rate = [c for c in counters if c.endswith("_SIZE")]
cols += [f"{c} TB/s" for c in rate]
if a.per:
    cols.append("us/step")
print("| " + " | ".join(cols) + " | kernel |")
print("|" + "---:|" * len(cols) + "---|")
for name, g in sorted(agg.items(), key=lambda kv: -kv[1]["ns"])[: a.n]:
    n = g["n"]
    cells = [str(n), f"{g['ns'] / n / 1e3:.2f}"] + [f"{g[c] / n:,.0f}" for c in counters]
    cells += [f"{g[c] * 1024 / max(1, g['ns']) / 1e3:.2f}" for c in rate]
    if a.per:
        cells.append(f"{g['ns'] / 1e3 / a.per:.1f}")
    print("| " + " | ".join(cells) + f" | `{name[:90]}` |")
