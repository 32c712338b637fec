# timed-window kernel table of the 70B TP=8 per-rank probe (round-4 tiles, fused exchange, batched merge)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tpp -o tp -- python3 $R/bench/tp_probe.py --preset llama3-70b --tp 8 --steps 1 --warmup 1 > gpurun_out/tpp.log 2>&1 || { tail -5 gpurun_out/tpp.log; exit 2; }
python3 scripts/prof_window.py $(find gpurun_out/tpp -name '*kernel_trace.csv' | head -1) "tp_probe 70B TP=8 rank 0, timed wave (round-4 tiles)" 30 --per 127 > gpurun_out/tpp_window.md
head -16 gpurun_out/tpp_window.md
rm -rf gpurun_out/tpp
