"""The tensor-parallel engine with N ranks sharing ONE GPU (gloo step protocol, one-shot IPC exchange fused into the
row-parallel GEMMs, hipGraph decode), checked token for token against TP=1 — the 8-rank case of
tests/test_engine_gpu.py::test_tensor_parallel_on_one_gpu, run from a parent that never touches the GPU (the test
runner's own context would be a 9th process on the card; its time-sliced queues stalled the 8-rank group's
spinning exchanges in round 6).

    python scripts/tp_ranks_one_gpu.py --world 8        # prints one JSON line; exit 0 iff tokens agree

The TP=1 reference (greedy no-cache recompute with the same full-size weights) runs in a child after the group has
exited. Greedy tokens must agree up to near-ties (tests/test_engine_gpu.py agree); every rank's device-side token rows are
compared (they advance on every rank when the group runs decode windows)."""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PROMPTS = [[5, 9, 33, 12, 7] * 9, [100, 200, 300], list(range(3, 140))]


def _group(rank, world, port, window, q):
    import torch
    import torch.distributed as dist

    from src.config import EngineConfig
    from src.parallel.tp import TPContext
    from src.parallel.tp_runner import build_tp_engine
    from src.preproc import SamplingParams

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tp = TPContext(rank=rank, world_size=world)
        cfg = EngineConfig(max_num_seqs=4, max_num_batched_tokens=256, num_kv_blocks=128, max_latency_ms=0.0,
                           use_cuda_graph=True, graph_batch_sizes=[1, 2, 4], decode_window=window)
        obj = build_tp_engine("llama-mini", tp, "cuda:0", cfg=cfg, max_model_len=512, capture=True, full_init=True,
                              seed=3)
        if rank == 0:
            obj.eos_token_id = None
            plan = obj.model.decode_plan(4)
            t0 = time.perf_counter()
            outs = obj.generate(PROMPTS, SamplingParams(max_tokens=8))
            el = time.perf_counter() - t0
            obj.runner.stop_followers()
            torch.cuda.synchronize()
            q.put((0, {"tokens": outs, "generate_s": round(el, 3), "error_word": bool(tp.car.error()),
                       "tp_fused": bool(plan["tp_fused"]), "o": list(plan["o"]), "down": list(plan["down"]),
                       "windows": obj.runner.windows_synced, "d_tokens": obj.runner.d_tokens.cpu().numpy()}))
        else:
            obj.follower_loop()
            torch.cuda.synchronize()
            q.put((rank, {"d_tokens": obj.d_tokens.cpu().numpy()}))
    finally:
        dist.destroy_process_group()


def _reference(q):
    from src.models.llama import CausalLM
    from src.models.presets import get_preset
    from tests.test_engine_gpu import reference_with_margins

    m = CausalLM(get_preset("llama-mini"), "cuda:0", seed=3, max_position=512, full_init=True)
    q.put([reference_with_margins(m, p, 8) for p in PROMPTS])


def main(argv=None) -> int:
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--window", type=int, default=8)
    a = ap.parse_args(argv)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_group, args=(r, a.world, port, a.window, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(a.world))
    for p in ps:
        p.join(60)
    lead = res[0]
    ranks_agree = all((res[r]["d_tokens"] == lead["d_tokens"]).all() for r in range(1, a.world))
    rq = ctx.Queue()
    rp = ctx.Process(target=_reference, args=(rq,))
    rp.start()
    refs = rq.get(timeout=300)
    rp.join(60)
    from tests.test_engine_gpu import agree

    tok_ok = all(agree(o, r, m) for o, (r, m) in zip(lead["tokens"], refs))
    out = {"check": "tp_ranks_one_gpu", "world": a.world, "window": a.window, "tokens_match_tp1": tok_ok,
           "ranks_agree": bool(ranks_agree), "exit_codes": [p.exitcode for p in ps],
           **{k: lead[k] for k in ("generate_s", "error_word", "tp_fused", "o", "down", "windows")}}
    print(json.dumps(out), flush=True)
    ok = tok_ok and ranks_agree and not lead["error_word"] and all(p.exitcode == 0 for p in ps)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
