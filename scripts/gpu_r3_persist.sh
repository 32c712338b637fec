# persistent decode-step kernel: bit-exactness vs the multi-launch path, then its speed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $T tests/test_decode_persistent_gpu.py -k intermediates > gpurun_out/r3p_inter.log 2>&1 || exit 1
timeout -k 10 400 $T tests/test_decode_persistent_gpu.py > gpurun_out/r3p_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench/micro_decode_persistent.py 32 20 > gpurun_out/r3p_bench.log 2>&1 || exit 2
