# round 3, first GPU check: the new failure-path / RCCL / served-length tests, the one-shot collective
# tests (healthy path unchanged), then the headline bench and the serving path through the coordinator
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "served_lengths or prefill" > gpurun_out/r3_kern.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_custom_allreduce_gpu.py tests/test_rccl_gpu.py tests/test_engine_gpu.py -k "allreduce or rccl or fails_as_a_unit" > gpurun_out/r3_tp.log 2>&1 || exit 2
timeout -k 10 900 $T tests/test_oracle_gpu.py > gpurun_out/r3_oracle.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r3_bench.log 2>&1 || exit 4
timeout -k 10 600 python bench/serve_bench.py --mode llm --gpus 1 --concurrency 32 > gpurun_out/r3_serve.log 2>&1 || exit 5
