# 70B TP=8 shard decode attention phases (engine qkv split 8 vs 2 slabs), 8B for comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for args in "--shape 70b_tp8" "--shape 70b_tp8 --sk 2" "--shape 70b_tp8 --sk 1" "--shape 8b --sk 1"; do
  timeout -k 10 120 python bench/micro_attn_timeline.py --ctx 576 $args > gpurun_out/tl70.log 2>&1 || { tail -5 gpurun_out/tl70.log; exit 4; }
  grep '^{' gpurun_out/tl70.log
done
