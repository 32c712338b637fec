# round 5 A/B: decode GEMM on tile-order weight copies (default) vs the row-major weights prefill also uses
# (DIE_GD_TILED=0), with and without the per-workgroup K-chunk rotation (DIE_GD_ROT=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_$name.log 2>&1 || { tail -5 gpurun_out/ab_$name.log; return 1; }
  echo "$name $(grep '^{' gpurun_out/ab_$name.log)"
}
run tiled_a DIE_GD_TILED=1 && run rot_a DIE_GD_TILED=0 DIE_GD_ROT=1 && run plain_a DIE_GD_TILED=0 DIE_GD_ROT=0 && \
run tiled_b DIE_GD_TILED=1 && run rot_b DIE_GD_TILED=0 DIE_GD_ROT=1
