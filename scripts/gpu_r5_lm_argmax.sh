#!/bin/bash
# LM head with per-tile greedy candidates (ops.linear_tiled_argmax + ops.sample(lm_part=...)): kernel tests, the
# engine / oracle tests, the micro A/B in graphs, the bench's timed-region kernel table and a bench run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "argmax or sample or gemm_decode or tiled or grouped or moe" > gpurun_out/r5_lmarg_tests.log 2>&1 || { tail -40 gpurun_out/r5_lmarg_tests.log; exit 1; }
tail -1 gpurun_out/r5_lmarg_tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_oracle_gpu.py tests/test_serving_gpu.py tests/test_expert_parallel_gpu.py > gpurun_out/r5_lmarg_tests2.log 2>&1 || { tail -40 gpurun_out/r5_lmarg_tests2.log; exit 1; }
tail -1 gpurun_out/r5_lmarg_tests2.log
timeout -k 10 120 python -u bench/micro_lm_head_argmax.py > gpurun_out/r5_lmarg_micro.jsonl 2>&1 || { tail -5 gpurun_out/r5_lmarg_micro.jsonl; exit 2; }
cat gpurun_out/r5_lmarg_micro.jsonl
export DIE_PROF_MARKERS=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/pa -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/r5_lmarg_prof.log 2>&1 || { tail -5 gpurun_out/r5_lmarg_prof.log; exit 3; }
T=$(find /tmp/pa -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_window.py $T "bench.py timed region (2 waves), LM head argmax candidates" 30 --per 254 > gpurun_out/r5_lmarg_window.md
unset DIE_PROF_MARKERS
timeout -k 10 300 python -u bench.py > gpurun_out/r5_lmarg_bench.log 2>&1 || { tail -5 gpurun_out/r5_lmarg_bench.log; exit 4; }
tail -n 1 gpurun_out/r5_lmarg_bench.log
grep -E "sample_kernel|gemm_decode_kernel<128, 0, 3|Timed window" gpurun_out/r5_lmarg_window.md
