#!/bin/bash
# sampling + decode input advance in one launch (ops.sample_advance): kernel equivalence test, engine / oracle /
# serving tests, bench, timed-window kernel table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "sample or argmax or embed" > gpurun_out/r5_sa_tests.log 2>&1 || { tail -40 gpurun_out/r5_sa_tests.log; exit 1; }
tail -1 gpurun_out/r5_sa_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_oracle_gpu.py tests/test_serving_gpu.py tests/test_bench_gpu.py > gpurun_out/r5_sa_tests2.log 2>&1 || { tail -40 gpurun_out/r5_sa_tests2.log; exit 1; }
tail -1 gpurun_out/r5_sa_tests2.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5_sa_bench.log 2>&1 || { tail -5 gpurun_out/r5_sa_bench.log; exit 2; }
grep '^{' gpurun_out/r5_sa_bench.log | cut -c1-200
export DIE_PROF_MARKERS=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/sa -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > gpurun_out/r5_sa_prof.log 2>&1 || { tail -5 gpurun_out/r5_sa_prof.log; exit 3; }
T=$(find /tmp/sa -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_window.py $T "bench.py timed region (2 waves), sampling + input advance + next embedding in one launch" 20 --per 254 > gpurun_out/r5_sa_window.md
grep -E "Timed window|sample_kernel|decode_advance|embed_sumsq|rmsnorm" gpurun_out/r5_sa_window.md
