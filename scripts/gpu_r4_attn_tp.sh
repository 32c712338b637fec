# dynamic attention split for TP shards: kernel/engine tests, TP probes, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_oracle_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/at_tests.log 2>&1 || { tail -30 gpurun_out/at_tests.log; exit 1; }
tail -1 gpurun_out/at_tests.log
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/at_tp70.log 2>&1 || exit 4
grep -h '^{' gpurun_out/at_tp70.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/at_tp8.log 2>&1 || exit 5
grep -h '^{' gpurun_out/at_tp8.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/at_bench.log 2>&1 || { tail -5 gpurun_out/at_bench.log; exit 3; }
grep '^{' gpurun_out/at_bench.log
