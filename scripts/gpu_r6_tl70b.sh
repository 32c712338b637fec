# 70B TP=8 shard decode attention: 2-chunk parts (max_ctx 2048, the engine's bound) vs 1-chunk parts (1024)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mc in 2048 1024 2048 1024; do
  timeout -k 10 120 python bench/micro_attn_timeline.py --ctx 576 --shape 70b_tp8 --max-ctx $mc > gpurun_out/tl70b.log 2>&1 || { tail -5 gpurun_out/tl70b.log; exit 4; }
  grep '^{' gpurun_out/tl70b.log
done
