# round 6: Llama-3-70B on ONE GPU with the swept row-major decode tiles: kernel tests at its shapes, the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "residual_mode or rownorm_silu or uneven" -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_70b_ktests.log 2>&1 || { tail -30 gpurun_out/r6_70b_ktests.log; exit 1; }
tail -1 gpurun_out/r6_70b_ktests.log
timeout -k 10 500 python -u bench.py --preset llama3-70b --steps 2 --warmup 1 > gpurun_out/r6_70b_bench2.log 2>&1 || { tail -20 gpurun_out/r6_70b_bench2.log; exit 2; }
grep '^{' gpurun_out/r6_70b_bench2.log | cut -c1-250
