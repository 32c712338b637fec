# breadth: batches above the decode kernels' 32 rows, and 8K-token prompts (not the headline config)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/br_b64.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/br_b128.log 2>&1 || exit 2
timeout -k 10 500 python bench.py --prompt-len 8192 --max-model-len 8448 --steps 1 --warmup 1 > gpurun_out/br_p8k.log 2>&1 || exit 3
