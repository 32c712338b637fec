# round 6: the TP exchange calibration (fused vs separate, forced on 2 ranks sharing the GPU) + TP engine tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "calibration or tensor_parallel or tp_group" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r6cal_tests.log 2>&1 || { echo "FAILED"; tail -40 gpurun_out/r6cal_tests.log; exit 2; }
grep -E "PASSED|FAILED" gpurun_out/r6cal_tests.log
timeout -k 10 200 python -u scripts/tp_ranks_one_gpu.py --world 8 > gpurun_out/r6cal_8ranks.log 2>&1 || { tail -20 gpurun_out/r6cal_8ranks.log; exit 3; }
grep -h '^{' gpurun_out/r6cal_8ranks.log
