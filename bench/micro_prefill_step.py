"""Cost of one prefill step as a function of its size: N prompts x L tokens through LLMEngine.generate
(max_tokens = 1: one prefill step + sampling), Llama-3-8B random init, wall time per step and per
token, GPU kernel time per step (torch.cuda events around the step), and the host-side share.
Small prefill steps are what continuous admission runs between decode windows (bench/poisson_bench.py).

    python bench/micro_prefill_step.py [L] [N ...]
"""
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from src.config import EngineConfig  # noqa: E402
from src.engine import LLMEngine  # noqa: E402
from src.preproc import SamplingParams  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    ns = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8, 32]
    cfg = EngineConfig(max_num_seqs=64, max_num_batched_tokens=32768, max_latency_ms=0.0)
    eng = LLMEngine.from_preset("llama3-8b", device=torch.device("cuda:0"), cfg=cfg, max_model_len=2048, seed=1)
    eng.eos_token_id = None
    vocab = eng.arch.vocab_size
    rng = random.Random(3)
    sp = SamplingParams(max_tokens=1, ignore_eos=True)
    for n in ns:
        for rep in range(4):  # 1 warm-up + 3 timed; fresh prompts (no prefix-cache hits)
            prompts = [[rng.randrange(3, vocab) for _ in range(L)] for _ in range(n)]
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            ev0.record()
            eng.generate(prompts, sp)
            ev1.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            gpu = ev0.elapsed_time(ev1)
            if rep:
                print(json.dumps({"bench": "prefill_step", "prompts": n, "len": L, "tokens": n * L,
                                  "wall_ms": round(wall, 2), "gpu_span_ms": round(gpu, 2),
                                  "us_per_token": round(wall * 1e3 / (n * L), 2)}), flush=True)


if __name__ == "__main__":
    main()
