# breadth: decode batches of 64 / 128 rows (64- and 128-row decode-GEMM images), 8K-token prompts, Mixtral-8x7B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --batch 64 --steps 2 --warmup 1 > gpurun_out/br_b64.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/br_b128.log 2>&1 || exit 2
[ -n "$NO_8K" ] || timeout -k 10 500 python bench.py --prompt-len 8192 --max-model-len 8448 --steps 1 --warmup 1 > gpurun_out/br_p8k.log 2>&1 || exit 3
[ -n "$NO_MOE" ] || timeout -k 10 500 python bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/br_mixtral.log 2>&1 || exit 4
for f in br_b64 br_b128 br_p8k br_mixtral; do [ -f gpurun_out/$f.log ] && { echo -n "$f "; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|rank0_decode_s": [0-9.]*\|rank0_prefill_s": [0-9.]*' gpurun_out/$f.log | tr '\n' ' '; echo; }; done
