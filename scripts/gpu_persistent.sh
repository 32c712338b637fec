# persistent decode step: GPU tests, micro bench against the five-launch layer (release build), per-phase
# timeline (diagnostics build: DIE_KERNEL_DIAG=1 python -m src._build -> src/_Cdiag, loaded with DIE_C_DIAG=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_persistent_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dp_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/dp_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 240 python -u bench/micro_decode_persistent.py 32 20 > gpurun_out/dp_micro.log 2>&1 || { tail -20 gpurun_out/dp_micro.log; exit 2; }
grep '^{' gpurun_out/dp_micro.log
DIE_C_DIAG=1 timeout -k 10 240 python -u bench/prof_decode_persistent.py 4 > gpurun_out/dp_diag.log 2>&1 || { tail -20 gpurun_out/dp_diag.log; exit 3; }
grep '^{' gpurun_out/dp_diag.log | grep -v '"wave"'
