#!/bin/bash
# PMC passes over the persistent decode-step kernel (4 layers of Llama-3-8B shapes, batch 32); one pass per
# run, counters within the per-block limits. Usage (GPU box): bash scripts/pmc_persistent.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM"
P2="SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA"
P3="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p$i -- python3 $R/bench/prof_decode_persistent.py 4 > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
find $OUT -name "*counter_collection*.csv" | sort
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(os.path.join(out, "**", "*counter_collection*.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "decode_persistent_kernel" not in row.get("Kernel_Name", ""):
            continue
        agg[row["Counter_Name"]] += float(row["Counter_Value"])
        n[row["Counter_Name"]] += 1
with open(os.path.join(out, "summary.txt"), "w") as fo:
    for k in sorted(agg):
        fo.write(f"{k} total={agg[k]:.4g} rows={n[k]}\n")
avail = open(os.path.join(out, "avail.txt")).read().splitlines()
with open(os.path.join(out, "avail_sq.txt"), "w") as fo:
    fo.write("\n".join(l for l in avail if "SQC_" in l or "SQ_I" in l or "SQ_WAIT" in l))
PY
find $OUT -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
rm -f $OUT/avail.txt
cat $OUT/summary.txt
