# round 4 rehearsal: full GPU suite, smoke, bench (10 waves), TP probes, overlapped disaggregation bench,
# 8B tile sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --deselect tests/test_custom_allreduce_gpu.py --deselect tests/test_decode_persistent_gpu.py --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/r4f_tests.log | head -20; tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -1 gpurun_out/r4f_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r4f_smoke.log 2>&1 || { tail -5 gpurun_out/r4f_smoke.log; exit 2; }
timeout -k 10 120 python bench/micro_attn_timeline.py > gpurun_out/r4f_attn_timeline.jsonl 2>&1 || exit 11
cat gpurun_out/r4f_attn_timeline.jsonl
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r4f_bench.log 2>&1 || { tail -5 gpurun_out/r4f_bench.log; exit 3; }
grep '^{' gpurun_out/r4f_bench.log
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r4f_tp70.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r4f_tp70.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r4f_tp8.log 2>&1 || exit 5
grep -h '^{' gpurun_out/r4f_tp8.log
timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/r4f_disagg.jsonl 2> gpurun_out/r4f_disagg.err || { tail -5 gpurun_out/r4f_disagg.err; exit 6; }
cat gpurun_out/r4f_disagg.jsonl
DIE_KV_OVERLAP=0 timeout -k 10 600 python -u bench/disagg_serve_bench.py --steps 3 --log-dir gpurun_out > gpurun_out/r4f_disagg_noov.jsonl 2>> gpurun_out/r4f_disagg.err || { tail -5 gpurun_out/r4f_disagg.err; exit 7; }
cat gpurun_out/r4f_disagg_noov.jsonl
timeout -k 10 500 python -u bench/micro_tp_tiles.py --shapes 8b > gpurun_out/r4f_8b_tiles.jsonl 2>&1 || exit 8
grep best gpurun_out/r4f_8b_tiles.jsonl
timeout -k 10 300 python -u bench/micro_prefill_tail.py > gpurun_out/r4f_prefill_tail.jsonl 2>&1 || exit 9
cat gpurun_out/r4f_prefill_tail.jsonl
DIE_PREFILL_RESID_GEMM=1 timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r4f_bench_resid.log 2>&1 || { tail -5 gpurun_out/r4f_bench_resid.log; exit 10; }
grep '^{' gpurun_out/r4f_bench_resid.log
