# round 5: timed-region kernel tables (DIE_PROF_MARKERS=1 + scripts/prof_window.py) of the driver bench (Llama-3-8B,
# 2 timed waves) and the TP shard probes (70B TP=8, 8B TP=2); traces stay in /tmp, the tables go to gpurun_out/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p5b -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/p5b.log 2>&1 || { tail -5 gpurun_out/p5b.log; exit 1; }
python3 scripts/prof_window.py $(find /tmp/p5b -name '*kernel_trace.csv' | head -1) "bench.py timed region (2 waves), round 5" 30 --per 254 > gpurun_out/p5b_window.md
head -14 gpurun_out/p5b_window.md
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p5t -o tp -- python3 $R/bench/tp_probe.py --preset llama3-70b --tp 8 --steps 1 --warmup 1 > gpurun_out/p5t.log 2>&1 || { tail -5 gpurun_out/p5t.log; exit 2; }
python3 scripts/prof_window.py $(find /tmp/p5t -name '*kernel_trace.csv' | head -1) "tp_probe 70B TP=8 rank 0, timed wave, round 5" 30 --per 127 > gpurun_out/p5t_window.md
head -14 gpurun_out/p5t_window.md
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p5s -o tp -- python3 $R/bench/tp_probe.py --preset llama3-8b --tp 2 --steps 1 --warmup 1 > gpurun_out/p5s.log 2>&1 || { tail -5 gpurun_out/p5s.log; exit 3; }
python3 scripts/prof_window.py $(find /tmp/p5s -name '*kernel_trace.csv' | head -1) "tp_probe 8B TP=2 rank 0, timed wave, round 5" 30 --per 127 > gpurun_out/p5s_window.md
head -14 gpurun_out/p5s_window.md
