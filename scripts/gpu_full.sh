set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/full_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/full_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/full_smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/full_bench.log 2>&1 || exit 3
timeout -k 10 900 python bench/serve_bench.py --mode llm --gpus 1 --concurrency 32 > gpurun_out/full_serve_llm.log 2>&1 || exit 4
