set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in 0 3 2 1; do
DIE_ATTN_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pma$d -o a -- python3 $R/bench/micro_attn_decode.py 32 512 640 > $R/gpurun_out/pma$d.log 2>&1 || exit 1
done
