# round 6: 8 ranks on one GPU vs TP=1, TP probes (windows + half-LDS ring) with a timed-window kernel table,
# config 5's balancer on real worker processes (GPU test + 8B bench), headline bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/tp_ranks_one_gpu.py --world 8 > gpurun_out/r6c_tp8ranks.log 2>&1 || { echo "8 RANKS FAILED"; tail -20 gpurun_out/r6c_tp8ranks.log; exit 7; }
grep -h '^{' gpurun_out/r6c_tp8ranks.log
timeout -k 10 400 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r6c_tp70.log 2>&1 || { tail -20 gpurun_out/r6c_tp70.log; exit 3; }
grep -h '^{' gpurun_out/r6c_tp70.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r6c_tp8.log 2>&1 || { tail -20 gpurun_out/r6c_tp8.log; exit 4; }
grep -h '^{' gpurun_out/r6c_tp8.log
DIE_PROF_MARKERS=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tpp -o tp -- python3 $R/bench/tp_probe.py --preset llama3-70b --tp 8 --steps 1 --warmup 1 > gpurun_out/r6c_tpp.log 2>&1 || { tail -5 gpurun_out/r6c_tpp.log; exit 8; }
python3 scripts/prof_window.py $(find gpurun_out/tpp -name '*kernel_trace.csv' | head -1) "tp_probe 70B TP=8 rank 0, timed wave (round 6: decode windows, half-LDS ring o/down)" 30 --per 127 > gpurun_out/r6c_tpp_window.md
head -16 gpurun_out/r6c_tpp_window.md
rm -rf gpurun_out/tpp
timeout -k 10 400 python -u -m pytest tests/test_serving_gpu.py -k "lb_serving" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6c_lb_test.log 2>&1 || { echo "LB TEST FAILED"; tail -40 gpurun_out/r6c_lb_test.log; exit 5; }
grep -E "PASSED|FAILED" gpurun_out/r6c_lb_test.log
timeout -k 10 600 python -u bench/lb_serving_bench.py --preset llama3-8b --workers 3 --slow 1 --requests 192 --concurrency 48 --kv-blocks 2048 > gpurun_out/r6c_lb_bench.log 2>&1 || { tail -20 gpurun_out/r6c_lb_bench.log; exit 6; }
grep -h '^{' gpurun_out/r6c_lb_bench.log | cut -c1-300
timeout -k 10 400 python bench.py > gpurun_out/r6c_bench.log 2>&1 || { tail -5 gpurun_out/r6c_bench.log; exit 9; }
grep '^{' gpurun_out/r6c_bench.log | cut -c1-400
