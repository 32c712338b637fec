# tests -> smoke -> bench; stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/rt_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/rt_tests.log; exit 1; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/rt_smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/rt_bench.log 2>&1 || exit 3
