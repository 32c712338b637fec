# round 6 final tree: timed-region kernel tables (headline bench, 8B TP=2 probe), config 2 over the RPC path, Poisson
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p6b -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/p6b.log 2>&1 || { tail -5 gpurun_out/p6b.log; exit 1; }
python3 scripts/prof_window.py $(find /tmp/p6b -name '*kernel_trace.csv' | head -1) "bench.py timed region (2 waves), round 6 final tree" 30 --per 254 > gpurun_out/p6b_window.md
head -14 gpurun_out/p6b_window.md
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p6s -o tp -- python3 $R/bench/tp_probe.py --preset llama3-8b --tp 2 --steps 1 --warmup 1 > gpurun_out/p6s.log 2>&1 || { tail -5 gpurun_out/p6s.log; exit 3; }
python3 scripts/prof_window.py $(find /tmp/p6s -name '*kernel_trace.csv' | head -1) "tp_probe 8B TP=2 rank 0, timed wave, round 6 (decode windows)" 30 --per 127 > gpurun_out/p6s_window.md
head -10 gpurun_out/p6s_window.md
unset DIE_PROF_MARKERS
timeout -k 10 600 python -u bench/serve_bench.py --mode llm --gpus 1 > gpurun_out/r6_serve_llm.log 2>&1 || { tail -10 gpurun_out/r6_serve_llm.log; exit 4; }
grep '^{' gpurun_out/r6_serve_llm.log | cut -c1-300
timeout -k 10 600 python -u bench/poisson_bench.py --rates 40 --modes auto --requests 300 > gpurun_out/r6_poisson.log 2>&1 || { tail -10 gpurun_out/r6_poisson.log; exit 5; }
grep '^{' gpurun_out/r6_poisson.log | cut -c1-300
