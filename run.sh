#!/usr/bin/env bash
# Launch a local deployment: one coordinator + N workers (the reference ships
# an empty run.sh). Workers register with the coordinator themselves.
#
#   ./run.sh                         # 2 mock echo workers on CPU (BASELINE config 1)
#   ARCH=llama PRESET=llama3-8b GPUS=8 ./run.sh      # one Llama-3-8B replica per MI355X
#   ARCH=llama PRESET=llama3-70b TP=8 ./run.sh       # one TP=8 group (torchrun) as one worker
#   DISAGG=1 ARCH=llama PRESET=llama3-8b ./run.sh    # prefill worker on GPU0 -> decode worker on GPU1
#     (PREFILL_GPU / DECODE_GPU pick the ordinals; both workers see every GPU and select theirs with --device,
#      so the prefill process can map the decode GPU's landing zone and write it over xGMI)
set -euo pipefail
cd "$(dirname "$0")"
ARCH=${ARCH:-mock}
PRESET=${PRESET:-llama3-8b}
MODEL=${MODEL:-$([ "$ARCH" = mock ] && echo echo || echo llama)}
GPUS=${GPUS:-2}
TP=${TP:-1}
PORT=${PORT:-9000}
STRATEGY=${STRATEGY:-least_latency}
LOGDIR=${LOGDIR:-/tmp/die-logs}
mkdir -p "$LOGDIR"
export HSA_ENABLE_IPC_MODE_LEGACY=0
[ "$ARCH" = mock ] || python -m src._build >/dev/null

pids=()
cleanup() { for p in "${pids[@]}"; do kill "$p" 2>/dev/null || true; done; }
trap cleanup EXIT INT TERM

python -m src.coordinator --listen-port "$PORT" --strategy "$STRATEGY" > "$LOGDIR/coordinator.log" 2>&1 &
pids+=($!)

if [ "${DISAGG:-0}" = 1 ]; then
  PREFILL_GPU=${PREFILL_GPU:-0}
  DECODE_GPU=${DECODE_GPU:-1}
  python -m src.worker --worker-id decode0 --port $((PORT + 2)) --model "$MODEL" --device "cuda:$DECODE_GPU" \
      --arch "$ARCH" --preset "$PRESET" --role decode > "$LOGDIR/decode0.log" 2>&1 &
  pids+=($!)
  python -m src.worker --worker-id prefill0 --port $((PORT + 1)) --model "$MODEL" --device "cuda:$PREFILL_GPU" \
      --arch "$ARCH" --preset "$PRESET" --role prefill --decode-worker 127.0.0.1:$((PORT + 2)) \
      --coordinator 127.0.0.1:$PORT > "$LOGDIR/prefill0.log" 2>&1 &
  pids+=($!)
elif [ "$TP" -gt 1 ]; then
  python -m torch.distributed.run --nnodes 1 --nproc-per-node "$TP" --master-addr 127.0.0.1 --master-port 29511 \
      -m src.parallel.tp_worker --worker-id tp0 --port $((PORT + 1)) --model "$MODEL" --arch "$ARCH" \
      --preset "$PRESET" --tp-size "$TP" --coordinator 127.0.0.1:$PORT > "$LOGDIR/tp0.log" 2>&1 &
  pids+=($!)
else
  for i in $(seq 0 $((GPUS - 1))); do
    HIP_VISIBLE_DEVICES=$i python -m src.worker --worker-id "w$i" --port $((PORT + 1 + i)) --model "$MODEL" \
        --arch "$ARCH" --preset "$PRESET" --coordinator 127.0.0.1:$PORT > "$LOGDIR/w$i.log" 2>&1 &
    pids+=($!)
  done
fi
echo "coordinator on 127.0.0.1:$PORT (logs in $LOGDIR); try:"
echo "  python examples/example_client.py --address 127.0.0.1:$PORT --model $MODEL $([ "$ARCH" = mock ] || echo --prompt hello)"
wait
