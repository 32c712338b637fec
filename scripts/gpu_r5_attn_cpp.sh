# round 5: single-chunk attention parts for few (sequence, kv head) pairs + prefill RMSNorm as row scales —
# tests, then the 70B TP=8 probe A/B and the bench A/B
# (the DIE_AB_* switches were temporary: removed once the A/B was recorded in profiles/r5_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode or row_scale or q_scale or silu or rope or attn_prefill" > gpurun_out/attn_cpp_tests.log 2>&1 || { tail -30 gpurun_out/attn_cpp_tests.log; exit 1; }
tail -3 gpurun_out/attn_cpp_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_oracle_gpu.py \
  > gpurun_out/attn_cpp_oracle.log 2>&1 || { tail -30 gpurun_out/attn_cpp_oracle.log; exit 1; }
tail -3 gpurun_out/attn_cpp_oracle.log
run() {  # name, cmd...
  local name=$1; shift
  env "$@" > gpurun_out/ab_$name.log 2>&1 || { tail -5 gpurun_out/ab_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab_$name.log | tail -1 | cut -c1-400)"
}
P="timeout -k 10 300 python bench/tp_probe.py"
B="timeout -k 10 300 python bench.py --steps 6 --warmup 2"
run tp_new_a X=1 $P && run tp_old_a DIE_AB_ATTN_OLD=1 $P && run tp_new_b X=1 $P && run tp_old_b DIE_AB_ATTN_OLD=1 $P && \
run pf_new_a X=1 $B && run pf_old_a DIE_AB_PF_OLD=1 $B && run pf_new_b X=1 $B && run pf_old_b DIE_AB_PF_OLD=1 $B
