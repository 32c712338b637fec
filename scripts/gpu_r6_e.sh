# round 6: same-box A/B of the TP probes (decode windows on/off, half-LDS ring vs round 5's full-ring tiles), then
# config 5 eviction with one weight layout vs the tile-order copies, and the prefill GEMM clock (PMC)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
for args in "--decode-window 8" "--decode-window 1" "--decode-window 8 --legacy-fused" "--decode-window 1 --legacy-fused" "--decode-window 8"; do
  timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 3 --warmup 1 $args > gpurun_out/r6e_tp70.log 2>&1 || { tail -20 gpurun_out/r6e_tp70.log; exit 3; }
  grep -h '^{' gpurun_out/r6e_tp70.log | tee -a gpurun_out/r6e_tp_ab.jsonl | cut -c1-330
done
for args in "--decode-window 8" "--decode-window 1"; do
  timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 3 --warmup 1 $args > gpurun_out/r6e_tp8.log 2>&1 || { tail -20 gpurun_out/r6e_tp8.log; exit 4; }
  grep -h '^{' gpurun_out/r6e_tp8.log | tee -a gpurun_out/r6e_tp_ab.jsonl | cut -c1-330
done
bash scripts/gpu_r6_d.sh
