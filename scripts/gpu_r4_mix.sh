# round 4: TP tests + probes after the tile sweep, overlapped disaggregated export (tests + two-process bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py tests/test_serving_gpu.py -k "allreduce or tensor_parallel or tp_group or export or disagg" -x -v --timeout 400 --timeout-method thread > gpurun_out/r4_mix_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r4_mix_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r4_mix_tests.log
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_70b_v2.log 2>&1 || exit 2
grep -h '^{' gpurun_out/r4_tp_probe_70b_v2.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_8b_v2.log 2>&1 || exit 3
grep -h '^{' gpurun_out/r4_tp_probe_8b_v2.log
timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/r4_disagg_overlap.jsonl 2> gpurun_out/r4_disagg2.err || { tail -5 gpurun_out/r4_disagg2.err; exit 4; }
cat gpurun_out/r4_disagg_overlap.jsonl
DIE_KV_OVERLAP=0 timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/r4_disagg_nooverlap.jsonl 2>> gpurun_out/r4_disagg2.err || { tail -5 gpurun_out/r4_disagg2.err; exit 5; }
cat gpurun_out/r4_disagg_nooverlap.jsonl
