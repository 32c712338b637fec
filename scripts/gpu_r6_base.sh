# round 6 baseline on this round's boxes: headline bench + the two TP probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r6b_bench.log 2>&1 || { tail -5 gpurun_out/r6b_bench.log; exit 3; }
grep '^{' gpurun_out/r6b_bench.log
timeout -k 10 400 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r6b_tp70.log 2>&1 || { tail -5 gpurun_out/r6b_tp70.log; exit 1; }
grep -h '^{' gpurun_out/r6b_tp70.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r6b_tp8.log 2>&1 || { tail -5 gpurun_out/r6b_tp8.log; exit 2; }
grep -h '^{' gpurun_out/r6b_tp8.log
