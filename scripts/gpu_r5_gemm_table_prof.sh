# round 5: kernel stats of the bench's prefill GEMMs with / without the prefill GEMM table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in table default; do
  extra=""; [ $v = default ] && extra="--no-gemm-table"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gt_$v -o run -- \
    python3 bench.py --steps 2 --warmup 1 $extra > gpurun_out/prof_gt_$v.log 2>&1 || { tail -5 gpurun_out/prof_gt_$v.log; exit 1; }
  f=$(find /tmp/prof_gt_$v -name '*kernel_trace.csv' | head -1)
  python - $f $v <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"]
    if "Cijk" in n or "rocblas" in n.lower() or "Rocblas" in n or "gemm" in n.lower() and "gemm_decode" not in n:
        g = (n[:90], r.get("Grid_Size_X", r.get("Grid_Size", "")))
        agg[g][0] += 1
        agg[g][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("#", sys.argv[2])
for (n, gx), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
    print(f"{t / 1e3:9.2f} ms {c:5d} calls {t / c:9.1f} us  grid {gx:>9}  {n}")
PY
done
