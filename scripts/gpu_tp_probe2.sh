# v3 merge area enlarged: fused-attention + engine tests, then the 70B TP=8 probe and the 8B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/tp2_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/tp_probe_70b_v2.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/tp2_bench.log 2>&1 || exit 3
