# round 4: TP decode with the one-shot exchange fused into the row-parallel GEMM's epilogue — the IPC
# collectives + fused GEMM at 2/4/8 ranks on the one GPU, the TP engine tests (token-exact vs TP=1, group
# fails as a unit), then the per-rank probe (70B TP=8, 8B TP=2) fused vs separate launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_rccl_gpu.py -k "tp_group or rccl or evicted" -x -v --timeout 400 --timeout-method thread > gpurun_out/r4_tp_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r4_tp_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r4_tp_tests.log
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_70b.log 2>&1 || exit 2
grep -h '^{' gpurun_out/r4_tp_probe_70b.log
DIE_TP_FUSED=0 timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_70b_sep.log 2>&1 || exit 3
grep -h '^{' gpurun_out/r4_tp_probe_70b_sep.log
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_8b.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r4_tp_probe_8b.log
DIE_TP_FUSED=0 timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/r4_tp_probe_8b_sep.log 2>&1 || exit 5
grep -h '^{' gpurun_out/r4_tp_probe_8b_sep.log
