# round 6: bisect the 8-rank TP engine test (windows vs the half-LDS ring exchange): IPC collectives at 8 ranks
# with the half ring at 4 and 19 rows, then the 8-rank engine test with the separate exchange, then fused
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_custom_allreduce_gpu.py -k "8" -x -v -s --timeout 150 --timeout-method thread > gpurun_out/r6_dbg_car.log 2>&1 || { echo "CAR FAILED"; tail -30 gpurun_out/r6_dbg_car.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r6_dbg_car.log
DIE_TP_FUSED=0 timeout -k 10 170 python -u -m pytest tests/test_engine_gpu.py -k "tensor_parallel and 8-True" -x -v -s --timeout 150 --timeout-method thread > gpurun_out/r6_dbg_tp8_sep.log 2>&1; echo "separate exit $?"
grep -E "PASSED|FAILED|Error|assert" gpurun_out/r6_dbg_tp8_sep.log | head -5
