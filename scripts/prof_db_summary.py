"""Summarise a rocprofv3 SQLite result (rocpd): per-kernel totals, plus wall-clock gaps.

python scripts/prof_db_summary.py <results.db> [title] [N]
"""
import sqlite3
import sys
from collections import defaultdict

db, title = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else sys.argv[1])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
c = sqlite3.connect(db)
rows = c.execute("select s.display_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
agg = defaultdict(lambda: [0, 0.0])
for name, s, e, gx, wx in rows:
    a = agg[name]
    a[0] += 1
    a[1] += (e - s)
tot = sum(v[1] for v in agg.values())
span = (rows[-1][2] - rows[0][1]) if rows else 0
print(f"# {title}\n\nTotal kernel time {tot / 1e6:.1f} ms over a {span / 1e6:.1f} ms span, {len(rows)} dispatches.\n")
print("| total ms | % | calls | avg us | kernel |\n|---:|---:|---:|---:|---|")
for name, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:n]:
    print(f"| {t / 1e6:.2f} | {100 * t / tot:.2f} | {cnt} | {t / cnt / 1e3:.2f} | `{name[:100]}` |")
