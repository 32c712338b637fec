set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/micro_decode_persistent.py 32 20 > gpurun_out/r3a_micro_dp.log 2>&1 || { tail -20 gpurun_out/r3a_micro_dp.log; exit 1; }
grep '^{' gpurun_out/r3a_micro_dp.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r3a_bench.log 2>&1 || { tail -20 gpurun_out/r3a_bench.log; exit 3; }
grep '^{' gpurun_out/r3a_bench.log
