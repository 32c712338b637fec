# 70B TP=8 shard probe at the serving bound (max_model_len 2,048): timed-window kernel table (few-pair attention split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export DIE_PROF_MARKERS=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8t -o tp -- python3 $R/bench/tp_probe.py --preset llama3-70b --tp 8 --steps 1 --warmup 1 --max-model-len 2048 > gpurun_out/p8t.log 2>&1 || { tail -5 gpurun_out/p8t.log; exit 1; }
python3 scripts/prof_window.py $(find /tmp/p8t -name '*kernel_trace.csv' | head -1) "tp_probe 70B TP=8 rank 0, timed wave at max_model_len 2,048 (few-pair attention split), round 6" 30 --per 127 > gpurun_out/p8t_window.md
head -14 gpurun_out/p8t_window.md
grep '^{' gpurun_out/p8t.log | cut -c1-300
