# round 6: TP windows + residency rule (tests, probes, 8 ranks on one GPU), then config 5's balancer on real workers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "custom_allreduce or tensor_parallel or tp_group or half_ring or refuses" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6b_tp_tests.log 2>&1 || { echo "TP TESTS FAILED"; tail -40 gpurun_out/r6b_tp_tests.log; exit 2; }
grep -cE "PASSED" gpurun_out/r6b_tp_tests.log
timeout -k 10 200 python -u scripts/tp_ranks_one_gpu.py --world 8 > gpurun_out/r6b_tp8ranks.log 2>&1 || { echo "8 RANKS FAILED"; tail -20 gpurun_out/r6b_tp8ranks.log; exit 7; }
grep -h '^{' gpurun_out/r6b_tp8ranks.log
timeout -k 10 400 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r6b_tp70.log 2>&1 || { tail -20 gpurun_out/r6b_tp70.log; exit 3; }
grep -h '^{' gpurun_out/r6b_tp70.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r6b_tp8.log 2>&1 || { tail -20 gpurun_out/r6b_tp8.log; exit 4; }
grep -h '^{' gpurun_out/r6b_tp8.log
timeout -k 10 400 python -u -m pytest tests/test_serving_gpu.py -k "lb_serving" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6b_lb_test.log 2>&1 || { echo "LB TEST FAILED"; tail -40 gpurun_out/r6b_lb_test.log; exit 5; }
grep -E "PASSED|FAILED" gpurun_out/r6b_lb_test.log
timeout -k 10 600 python -u bench/lb_serving_bench.py --preset llama3-8b --workers 3 --slow 1 --requests 192 --concurrency 48 --kv-blocks 2048 > gpurun_out/r6b_lb_bench.log 2>&1 || { tail -20 gpurun_out/r6b_lb_bench.log; exit 6; }
grep -h '^{' gpurun_out/r6b_lb_bench.log | cut -c1-400
