# round 5: prefill GEMM solution table (TunableOp, read-only) — test, then bench A/B on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_table or attn_prefill or gemm_decode_tiled" > gpurun_out/gt_tests.log 2>&1 || { tail -30 gpurun_out/gt_tests.log; exit 1; }
tail -2 gpurun_out/gt_tests.log
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 "$@" > gpurun_out/gt_$name.log 2>&1 || { tail -5 gpurun_out/gt_$name.log; return 1; }
  python - gpurun_out/gt_$name.log $name <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
n = d['notes']
print(sys.argv[2], d['value'], 'req/s; prefill', round(n['rank0_prefill_s'] / d['steps'] * 1e3, 1), 'ms/wave; decode',
      round(n['rank0_decode_s'] / d['steps'] / 127 * 1e3, 3), 'ms/step')
PY
}
run table_a && run default_a --no-gemm-table && run table_b && run default_b --no-gemm-table
