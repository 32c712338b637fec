# kernel-argument warm-up: decode kernel tests + oracle, attention timeline, bench (timed window profile)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_oracle_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ka_tests.log 2>&1 || { tail -30 gpurun_out/ka_tests.log; exit 1; }
tail -1 gpurun_out/ka_tests.log
timeout -k 10 120 python bench/micro_attn_timeline.py > gpurun_out/ka_attn_timeline.jsonl 2>&1 || exit 2
cat gpurun_out/ka_attn_timeline.jsonl
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/ka_bench.log 2>&1 || { tail -5 gpurun_out/ka_bench.log; exit 3; }
grep '^{' gpurun_out/ka_bench.log
R=$GRAFT_REPO_ROOT
DIE_PROF_MARKERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kap -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/ka_prof.log 2>&1 || { tail -5 gpurun_out/ka_prof.log; exit 4; }
python3 scripts/prof_window.py $(find gpurun_out/kap -name '*kernel_trace.csv' | head -1) "bench.py timed region (2 waves), kernel args warmed" 30 --per 254 > gpurun_out/ka_window.md
head -20 gpurun_out/ka_window.md
rm -rf gpurun_out/kap
