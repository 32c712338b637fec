# kernel tests -> engine tests -> bench -> profile; stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/it_tests.log 2>&1 || { echo "TESTS FAILED" >> gpurun_out/it_tests.log; exit 1; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/it_bench.log 2>&1 || exit 2
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/itprof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/it_prof.log 2>&1 || exit 3
