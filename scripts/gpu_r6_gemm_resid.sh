# prefill o / down with the residual add in the GEMM epilogue: numerics, then bench A/B on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "linear_residual or gemm_residual or row_scale" --timeout 120 --timeout-method thread > gpurun_out/gr_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gr_tests.log; exit 1; }
tail -2 gpurun_out/gr_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/gr_on_$i.log 2>&1 || { tail -5 gpurun_out/gr_on_$i.log; exit 3; }
  grep '^{' gpurun_out/gr_on_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('on ', d['value'], d['notes']['rank0_prefill_s'], d['notes']['rank0_decode_s'])"
  timeout -k 10 300 python bench.py --no-gemm-residual > gpurun_out/gr_off_$i.log 2>&1 || { tail -5 gpurun_out/gr_off_$i.log; exit 3; }
  grep '^{' gpurun_out/gr_off_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('off', d['value'], d['notes']['rank0_prefill_s'], d['notes']['rank0_decode_s'])"
done
# decode attention phase timelines at a bench-wave context (where the 8B and 70B TP=8 attention time goes)
timeout -k 10 120 python bench/micro_attn_timeline.py --ctx 576 > gpurun_out/gr_tl_8b.log 2>&1 || { tail -5 gpurun_out/gr_tl_8b.log; exit 4; }
tail -6 gpurun_out/gr_tl_8b.log
timeout -k 10 120 python bench/micro_attn_timeline.py --ctx 576 --shape 70b_tp8 > gpurun_out/gr_tl_70b.log 2>&1 || { tail -5 gpurun_out/gr_tl_70b.log; exit 4; }
tail -6 gpurun_out/gr_tl_70b.log
