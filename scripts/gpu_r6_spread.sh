# decode attention below one (sequence, kv head) pair per CU (8B TP=2: 128 pairs; 8B at batch 16): parts sized for
# two workgroups per CU ("spread") vs the static split — numerics, timelines, 8B TP=2 probe at bounds 2,048 and 704
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attn" --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/sp_tests.log; exit 1; }
tail -1 gpurun_out/sp_tests.log
for args in "--shape 8b_tp2" "--shape 8b_tp2 --spread" "--shape 8b --batch 16" "--shape 8b --batch 16 --spread" "--shape 8b" "--shape 8b --spread"; do
  timeout -k 10 120 python bench/micro_attn_timeline.py --ctx 576 $args > gpurun_out/sp_tl.log 2>&1 || { tail -5 gpurun_out/sp_tl.log; exit 2; }
  echo "$args $(grep '^{' gpurun_out/sp_tl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['workgroups_with_a_task'], d['span'], d['first_chunk'], d['stream'], d['merge_out'], d['tail'])")"
done
for mml in 2048 704; do
  for arg in "" "--attn-spread" "" "--attn-spread"; do
    timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 --max-model-len $mml $arg > gpurun_out/sp_tp.log 2>&1 || { tail -5 gpurun_out/sp_tp.log; exit 3; }
    grep -h '^{' gpurun_out/sp_tp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tp2 $mml', '$arg' or 'default', d['decode_ms_per_step'])"
  done
done
