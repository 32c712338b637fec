set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_engine_gpu.py -k "allreduce or tensor_parallel" -x -q --timeout 280 --timeout-method thread > gpurun_out/carm_test.log 2>&1 &&
DIE_CAR_MODE=0 timeout -k 10 200 python bench/micro_allreduce.py > gpurun_out/carm0.jsonl 2>/dev/null &&
DIE_CAR_MODE=1 timeout -k 10 200 python bench/micro_allreduce.py > gpurun_out/carm1.jsonl 2>/dev/null &&
DIE_CAR_MODE=3 timeout -k 10 200 python bench/micro_allreduce.py > gpurun_out/carm3.jsonl 2>/dev/null
