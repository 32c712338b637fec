# round 5: decode-attention timelines at the bench's and the 70B TP=8 rank's shapes, equal contexts (a wave)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { timeout -k 10 120 python bench/micro_attn_timeline.py "$@" 2>/dev/null | grep '^{' >> gpurun_out/r5_attn_tl.jsonl || return 1; }
: > gpurun_out/r5_attn_tl.jsonl
run --shape 8b --ctx 520 && run --shape 8b --ctx 576 && run --shape 8b --ctx 640 && run --shape 8b && \
run --shape 70b_tp8 --ctx 576 && run --shape 70b_tp8 --ctx 576 --max-ctx 640 && run --shape 70b_tp8 --ctx 576 --max-ctx 1024 && \
run --shape 70b_tp8 --ctx 576 --max-ctx 320
cat gpurun_out/r5_attn_tl.jsonl
