# round-4 final: the driver's exact steps, then the 8B 64/128-row tile candidates of the round-4 sweep in the graph
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4_driver_rehearsal.sh || exit $?
timeout -k 10 300 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/fin_b128.log 2>&1 || exit 11
DIE_TILE_OVERRIDE="4096,14336,3,128=64,64,4" timeout -k 10 300 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/fin_b128_down.log 2>&1 || exit 12
timeout -k 10 300 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/fin_b64.log 2>&1 || exit 13
DIE_TILE_OVERRIDE="4096,4096,3,64=32,256,2" timeout -k 10 300 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/fin_b64_o.log 2>&1 || exit 14
for f in fin_b128 fin_b128_down fin_b64 fin_b64_o; do echo -n "$f "; grep -o '"value": [0-9.]*\|rank0_decode_s": [0-9.]*' gpurun_out/$f.log | tr '\n' ' '; echo; done
