# prefill FFN in token blocks with SiLU * up on a side stream: numerics, then bench A/B (split 1 / 2 / 4) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm_residual or linear_residual" --timeout 120 --timeout-method thread > gpurun_out/fs_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/fs_tests.log; exit 1; }
tail -2 gpurun_out/fs_tests.log
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['notes']['rank0_prefill_s'], d['notes']['rank0_decode_s'])"; }
for i in 1 2; do
  for sp in 1 2 4; do  # interleaved
    timeout -k 10 300 python bench.py --ffn-split $sp > gpurun_out/fs_${sp}_$i.log 2>&1 || { tail -5 gpurun_out/fs_${sp}_$i.log; exit 3; }
    show gpurun_out/fs_${sp}_$i.log "split$sp"
  done
done
