# per-rank compute of TP configurations on one GPU (bench/tp_probe.py): 70B TP=8 (config 4), 8B TP=2;
# FULL=1 runs the whole GPU test suite first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tp_full_tests.log 2>&1 || { tail -30 gpurun_out/tp_full_tests.log; exit 4; }
  tail -1 gpurun_out/tp_full_tests.log
fi
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/tp_probe_70b.log 2>&1 || exit 1
grep -h '^{' gpurun_out/tp_probe_70b.log
DIE_GD_SILU_SPLITK=0 timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/tp_probe_70b_fullk.log 2>&1 || exit 2
grep -h '^{' gpurun_out/tp_probe_70b_fullk.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/tp_probe_8b.log 2>&1 || exit 3
