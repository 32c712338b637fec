set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DIE_KV_ZONE_BYTES=536870912 timeout -k 10 100 python -u scripts/repro_ipc_kv.py > gpurun_out/repro_kv_512.log 2>&1 ; echo "rc $?" >> gpurun_out/repro_kv_512.log
DIE_KV_ZONE_BYTES=1073741824 timeout -k 10 100 python -u scripts/repro_ipc_kv.py > gpurun_out/repro_kv_1g.log 2>&1; echo "rc $?" >> gpurun_out/repro_kv_1g.log
