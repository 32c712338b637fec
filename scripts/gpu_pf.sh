# prefill attention: NS=1 vs NS=2 stages, numerics then micro
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "prefill or attention" --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || exit 1
for ns in 1 2; do
  DIE_PF_NS=$ns timeout -k 10 120 python -u bench/micro_attn_prefill.py 32 512 >> gpurun_out/pf_micro.jsonl 2>/dev/null || exit 2
  DIE_PF_NS=$ns timeout -k 10 120 python -u bench/micro_attn_prefill.py 4 4096 >> gpurun_out/pf_micro.jsonl 2>/dev/null || exit 3
done
