# the node-section rehearsal on its own, output streamed to gpurun_out (debugging a stall)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 150 python bench.py --gpus 2 --same-device --preset llama-mini --batch 8 --prompt-len 64 --gen-len 16 --max-model-len 256 --steps 1 --warmup 1 --tp-wave-min-world 2 --tp-wave-preset llama-mini --cross-gpu-budget-s 100 --verbose > gpurun_out/r5_node_dbg.out 2> gpurun_out/r5_node_dbg.err
echo "rc=$?"
grep -v amdgpu.ids gpurun_out/r5_node_dbg.err | tail -30
cat gpurun_out/r5_node_dbg.out | head -c 3000
