"""Summarise a rocprofv3 kernel_stats.csv: python scripts/prof_summary.py <csv> [title] [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
title = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# {title}\n\nTotal kernel time {tot/1e6:.1f} ms.\n")
print("| total ms | % | calls | avg us | kernel |\n|---:|---:|---:|---:|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"| {float(r['TotalDurationNs'])/1e6:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
          f"{float(r['AverageNs'])/1e3:.2f} | `{r['Name'][:100]}` |")
