# mixed prefill/decode steps: GPU engine tests, then the open-loop Poisson serving bench (8B):
# 512-token prompts (the headline shape) and 32-token prompts (short chat turns)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mx_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/mx_tests.log; exit 1; }
timeout -k 10 500 python bench/poisson_bench.py --rates ${RATES:-20,30,40} --requests ${NREQ:-200} --modes auto,off,always > gpurun_out/poisson.jsonl 2> gpurun_out/poisson.err || { echo "POISSON FAILED"; tail -5 gpurun_out/poisson.err; exit 2; }
timeout -k 10 400 python bench/poisson_bench.py --rates 40,80 --requests 300 --prompt-len 32 --modes auto,off > gpurun_out/poisson_short.jsonl 2> gpurun_out/poisson_short.err || { echo "POISSON SHORT FAILED"; tail -5 gpurun_out/poisson_short.err; exit 3; }
python - <<'PY'
import json
for f in ("gpurun_out/poisson.jsonl", "gpurun_out/poisson_short.jsonl"):
    for l in open(f):
        d = json.loads(l)
        if "mode" in d:
            print(f.split("/")[-1], d["prompt_len"], d["mode"], d["rate_rps"], "rps", d["achieved_rps"], "ttft", d["ttft_ms"], "tpot", d["tpot_ms"], "x", d["tpot_p99_over_decode_step"], d["steps"])
        else:
            print(d)
PY
