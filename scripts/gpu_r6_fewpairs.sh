# decode attention for few (sequence, kv head) pairs: one chunk per part, one workgroup per task (up to 2 per CU)
# vs the static split — numerics, micro timeline, and the 70B TP=8 shard probe at the serving bound (2,048)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -k "attn or tensor_parallel or decode" --timeout 200 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/fp_tests.log; exit 1; }
tail -2 gpurun_out/fp_tests.log
for arg in "" "--static-parts"; do
  timeout -k 10 120 python bench/micro_attn_timeline.py --ctx 576 --shape 70b_tp8 $arg > gpurun_out/fp_tl.log 2>&1 || { tail -5 gpurun_out/fp_tl.log; exit 2; }
  grep '^{' gpurun_out/fp_tl.log | cut -c1-330
done
for i in 1 2; do
  for arg in "" "--attn-static-parts"; do
    timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 --max-model-len 2048 $arg > gpurun_out/fp_tp.log 2>&1 || { tail -5 gpurun_out/fp_tp.log; exit 3; }
    grep -h '^{' gpurun_out/fp_tp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arg' or 'few', d['decode_ms_per_step'], d['prefill_ms_per_wave'])"
  done
done
