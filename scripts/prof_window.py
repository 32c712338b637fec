"""Per-kernel table of a bench's TIMED region from a rocprofv3 kernel trace: keeps the dispatches between the
first and the last `spin_kernel` marker (benches launch them with DIE_PROF_MARKERS=1, src/utils/tracing.py
prof_marker) and drops model init, weight packing and warm-up.

    python scripts/prof_window.py <kernel_trace.csv> [title] [N] [--per STEPS]

--per: also divide each kernel's total by STEPS (e.g. decode steps) to give time per step."""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("title", nargs="?", default=None)
ap.add_argument("n", nargs="?", type=int, default=30)
ap.add_argument("--per", type=float, default=0.0)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[key]]
if len(marks) < 2:
    raise SystemExit(f"need two spin_kernel markers in {a.csv}, found {len(marks)} (run with DIE_PROF_MARKERS=1)")
win = rows[marks[0] + 1: marks[-1]]
t0, t1 = int(rows[marks[0]]["End_Timestamp"]), int(rows[marks[-1]]["Start_Timestamp"])
agg = defaultdict(lambda: [0, 0])
for r in win:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[r[key]][0] += d
    agg[r[key]][1] += 1
busy = sum(v[0] for v in agg.values())
print(f"# {a.title or a.csv}\n")
print(f"Timed window {(t1 - t0) / 1e6:.1f} ms between the markers; kernel-busy {busy / 1e6:.1f} ms "
      f"({100 * busy / max(1, t1 - t0):.1f} %), {len(win)} dispatches.\n")
hdr = "| total ms | % busy | calls | avg us |" + (" us per step |" if a.per else "") + " kernel |"
print(hdr + "\n|" + "---:|" * (hdr.count("|") - 2) + "---|")
for name, (tot, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.n]:
    per = f" {tot / 1e3 / a.per:.1f} |" if a.per else ""
    print(f"| {tot / 1e6:.2f} | {100 * tot / busy:.2f} | {n} | {tot / n / 1e3:.2f} |{per} `{name[:110]}` |")
