set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/it_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/it_tests.log; exit 1; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/it_bench.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --preset mixtral-8x7b > gpurun_out/it_bench_mixtral.log 2>&1 || exit 3
timeout -k 10 900 python bench/serve_bench.py --mode llm --gpus 1 --concurrency 32 > gpurun_out/it_serve_llm.log 2>&1 || exit 4
