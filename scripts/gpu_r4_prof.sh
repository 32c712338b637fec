# timed-region kernel tables (DIE_PROF_MARKERS=1 + scripts/prof_window.py): the driver bench (Llama-3-8B,
# 2 timed waves) and the TP shard probes (70B TP=8, 8B TP=2; fused row-parallel epilogue)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/p4b -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/p4b.log 2>&1 || { tail -5 gpurun_out/p4b.log; exit 1; }
python3 scripts/prof_window.py $(find gpurun_out/p4b -name '*kernel_trace.csv' | head -1) "bench.py timed region (2 waves)" 30 --per 254 > gpurun_out/p4b_window.md
head -12 gpurun_out/p4b_window.md
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/p4t -o tp -- python3 $R/bench/tp_probe.py --preset llama3-70b --tp 8 --steps 1 --warmup 1 > gpurun_out/p4t.log 2>&1 || { tail -5 gpurun_out/p4t.log; exit 2; }
python3 scripts/prof_window.py $(find gpurun_out/p4t -name '*kernel_trace.csv' | head -1) "tp_probe 70B TP=8 rank 0, timed wave" 30 --per 127 > gpurun_out/p4t_window.md
head -14 gpurun_out/p4t_window.md
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/p4s -o tp -- python3 $R/bench/tp_probe.py --preset llama3-8b --tp 2 --steps 1 --warmup 1 > gpurun_out/p4s.log 2>&1 || { tail -5 gpurun_out/p4s.log; exit 3; }
python3 scripts/prof_window.py $(find gpurun_out/p4s -name '*kernel_trace.csv' | head -1) "tp_probe 8B TP=2 rank 0, timed wave" 30 --per 127 > gpurun_out/p4s_window.md
rm -rf gpurun_out/p4b gpurun_out/p4t gpurun_out/p4s
