#!/usr/bin/env python3
"""
Headline benchmark (BASELINE.json): req/s + p50 end-to-end latency of
Llama-3-8B batched serving on 1/2/4/8 MI355X.

Each rank (one per GPU, launched by torch.distributed.run for N > 1) runs a
full serving replica — data parallel, the right layout for an 8B model that
fits one 288 GB GPU many times over — and the whole serving path minus TCP:

    Batcher(max_batch=32, max_latency=10 ms)  →  AsyncLLMEngine (engine thread)
      → continuous-batching scheduler → paged-KV Llama-3-8B (random-init bf16)
      → hand-written gfx950 kernels + hipBLASLt GEMMs, hipGraph decode.

One "step" = one wave of ``--batch`` (32) synthetic requests per GPU, each a
distinct random 512-token prompt generating 128 tokens (ignore_eos), submitted
together and served to completion (prefill + 128 decode iterations, sampling
included). Weak scaling: per-GPU work is fixed as N grows. ``value`` is the
whole-job request rate (all GPUs); ``p50_latency_ms`` is the median
submit→finish latency over every timed request.

    python bench.py                      # 1 GPU, 3 timed steps, 1 warmup
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 3 --warmup 1
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC_FMT = "req/sec + p50 end-to-end latency, {model} batched serving at 1/2/4/8 MI355X"


def model_label(preset: str) -> str:
    """Display name of a preset: llama3-8b -> Llama-3-8B, mixtral-8x7b -> Mixtral-8x7B."""
    from src.models.presets import get_preset

    name = getattr(get_preset(preset), "name", None) or preset
    if name.startswith("llama3"):
        name = "Llama-3" + name[len("llama3"):]
    elif name.startswith("mixtral"):
        name = "Mixtral" + name[len("mixtral"):]
    return name.replace("-8b", "-8B").replace("-70b", "-70B").replace("x7b", "x7B")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--batch", type=int, default=32, help="requests per GPU per step (= max_batch)")
    p.add_argument("--prompt-len", type=int, default=512)
    p.add_argument("--gen-len", type=int, default=128)
    p.add_argument("--preset", default="llama3-8b")
    p.add_argument("--max-latency-ms", type=float, default=10.0)
    p.add_argument("--max-model-len", type=int, default=2048)
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-async-decode", action="store_true", help="synchronous decode windows (A/B)")
    p.add_argument("--temperature", type=float, default=0.0)
    p.add_argument("--decode-window", type=int, default=None, help="decode steps per hipGraph window (engine default)")
    p.add_argument("--tp", type=int, default=1, help="tensor-parallel degree per replica (70B: --tp 8)")
    p.add_argument("--moe-parallel", choices=["tp", "ep"], default="tp", help="MoE layout under --tp")
    p.add_argument("--sequence-parallel", action="store_true", help="Megatron-SP prefill under --tp")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: reference-op engine over gloo (tests the multi-rank plumbing, not a measurement)")
    p.add_argument("--verbose", action="store_true")
    return p.parse_args()


def make_prompts(rng, n, prompt_len, vocab):
    """One wave's synthetic prompts (client-side data, generated before the clock starts)."""
    return [[rng.randrange(3, vocab) for _ in range(prompt_len)] for _ in range(n)]


async def serve_wave(batcher, prompts, gen_len, temperature):
    n = len(prompts)
    t0 = [0.0] * n
    lat = [0.0] * n

    async def one(i):
        t0[i] = time.perf_counter()
        fut = await batcher.add_request("llama", "1", {
            "prompt_token_ids": prompts[i], "max_tokens": gen_len, "ignore_eos": True,
            "temperature": temperature, "seed": i})
        seq = await fut
        lat[i] = time.perf_counter() - t0[i]
        assert len(seq.output_ids) == gen_len, (len(seq.output_ids), seq.finish_reason)

    await asyncio.gather(*(one(i) for i in range(n)))
    return lat


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = args.gpus or world
    on_gpu = args.device == "cuda"
    if world > 1:
        if on_gpu:
            torch.cuda.set_device(local)
        dist.init_process_group("nccl" if on_gpu else "gloo")  # nccl = RCCL over xGMI
    dev = torch.device(f"cuda:{local}" if on_gpu else "cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)

    from src.batcher import Batcher
    from src.config import EngineConfig
    from src.engine import LLMEngine
    from src.engine.async_engine import AsyncLLMEngine
    from src.preproc import normalize_request
    from src.utils.tracing import prof_marker

    cfg = EngineConfig(max_num_seqs=args.batch, max_num_batched_tokens=max(16384, args.prompt_len),
                       max_latency_ms=args.max_latency_ms, use_cuda_graph=not args.no_graph,
                       graph_batch_sizes=[1, 2, 4, 8, 16, 24, 32, args.batch],
                       async_decode=not args.no_async_decode,
                       **({"decode_window": args.decode_window} if args.decode_window else {}))
    t_init = time.perf_counter()
    tp = None
    if args.tp > 1:
        from src.parallel.tp import init_tp
        from src.parallel.tp_runner import build_tp_engine

        tp = init_tp(args.tp)
        obj = build_tp_engine(args.preset, tp, dev, cfg=cfg, max_model_len=args.max_model_len, seed=1234,
                              capture=not args.no_graph, moe_parallel=args.moe_parallel,
                              sequence_parallel=args.sequence_parallel)
        if tp.rank != 0:  # follower: mirror the leader through warmup and the timed waves
            obj.follower_loop()
            sync()
            dist.barrier()
            obj.follower_loop()
            sync()
            dist.barrier()
            t = torch.zeros(1, device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_gather_object([None] * world, 0.0)  # the leader's per-rank elapsed
            dist.all_gather_object([None] * world, [])
            dist.barrier()
            dist.destroy_process_group()
            return
        engine = obj
    else:
        engine = LLMEngine.from_preset(args.preset, device=dev, cfg=cfg, max_model_len=args.max_model_len,
                                       seed=1234, capture=not args.no_graph)
    engine.eos_token_id = None
    replicas = n_gpus // args.tp
    init_s = time.perf_counter() - t_init
    aeng = AsyncLLMEngine(engine)
    aeng.start()

    async def callback(model, version, inputs_list):
        loop = asyncio.get_running_loop()
        futs = []
        for x in inputs_list:
            gi = normalize_request(x, None, engine.max_model_len)
            futs.append(aeng.submit(os.urandom(8).hex(), gi.prompt_token_ids, gi.sampling, loop))
        return futs

    rng = random.Random(1000 + rank)

    async def run():
        batcher = Batcher(max_batch_size=args.batch, max_latency_ms=args.max_latency_ms, batch_callback=callback)
        await batcher.start()
        vocab = engine.arch.vocab_size
        for w in range(args.warmup):
            await serve_wave(batcher, make_prompts(rng, args.batch, args.prompt_len, vocab), args.gen_len,
                             args.temperature)
        waves = [make_prompts(rng, args.batch, args.prompt_len, vocab) for _ in range(args.steps)]
        sync()
        if tp is not None:
            engine.runner.stop_followers()
        if world > 1:
            dist.barrier()
        sync()
        prof_marker()
        stats0 = dict(engine.stats)
        t0 = time.perf_counter()
        lats = []
        for s in range(args.steps):
            lats += await serve_wave(batcher, waves[s], args.gen_len, args.temperature)
            if args.verbose and rank == 0:
                print(f"step {s}: {time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)
        prof_marker()
        sync()
        if tp is not None:
            engine.runner.stop_followers()
        if world > 1:
            dist.barrier()
        sync()
        elapsed = time.perf_counter() - t0
        await batcher.stop()
        return elapsed, lats, stats0

    elapsed, lats, stats0 = asyncio.run(run())
    aeng.stop()
    st = engine.stats
    gen_tok = st["generated_tokens"] - stats0["generated_tokens"]
    prefill_s = st["prefill_time"] - stats0["prefill_time"]
    decode_s = st["decode_time"] - stats0["decode_time"]
    rank_elapsed = [elapsed]
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rank_elapsed = [None] * world
        dist.all_gather_object(rank_elapsed, elapsed)
        elapsed = float(t.item())
        gathered = [None] * world
        dist.all_gather_object(gathered, lats)
        lats = [x for g in gathered for x in g]
    total_req = args.steps * args.batch * replicas
    rps = total_req / elapsed
    res = None
    if rank == 0:
        label = model_label(args.preset)
        res = {
            "metric": METRIC_FMT.format(model=label),
            "value": round(rps, 3),
            "unit": "req/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "p50_latency_ms": round(1e3 * statistics.median(lats), 2),
            "p99_latency_ms": round(1e3 * sorted(lats)[max(0, int(0.99 * len(lats)) - 1)], 2),
            "output_tok_per_s": round(gen_tok * replicas / elapsed, 1),
            "config": {
                "model": label,
                "global_batch": args.batch * replicas,
                "seq_len": args.prompt_len + args.gen_len,
                "prompt_len": args.prompt_len,
                "gen_len": args.gen_len,
                "parallelism": f"dp{replicas}" + (f"-tp{args.tp}" if args.tp > 1 else "")
                + ("-ep" if args.tp > 1 and args.moe_parallel == "ep" else "")
                + ("-sp" if args.tp > 1 and args.sequence_parallel else ""),
                "max_batch": args.batch,
                "max_latency_ms": args.max_latency_ms,
                "weights": "random-init",
                "hip_graph_decode": not args.no_graph,
            },
            "notes": {
                "baseline": "reference publishes no numbers and has no GPU path (BASELINE.md); vs_baseline=null",
                "rank0_prefill_s": round(prefill_s, 3),
                "rank0_decode_s": round(decode_s, 3),
                "engine_init_s": round(init_s, 1),
            },
        }
        if world > 1 and tp is None:  # the value uses the slowest replica; the spread shows stragglers
            res["notes"]["rank_elapsed_s"] = [round(x, 3) for x in rank_elapsed]
    dog = None
    if world > 1 and on_gpu and tp is None and os.environ.get("DIE_XGPU_PROBE", "1") != "0":
        # after the timed region: RCCL / one-shot IPC all-reduce / landing-zone KV hop between the real GPUs
        # (src/parallel/xgpu_probe.py), reported in notes. A watchdog armed until the process group is gone
        # prints the result without the probe (once) and ends the rank if anything after the timed region stalls.
        dog = _Watchdog(res, rank, 300.0)
        try:
            from src.parallel.xgpu_probe import xgpu_probe

            probe = xgpu_probe(rank, world, dev)
        except Exception as e:  # noqa: BLE001 — the bench result stands on its own
            probe = {"error": str(e)[:200]}
        if rank == 0:
            res["notes"]["xgpu_probe"] = probe
    if rank == 0:
        if dog is not None:
            dog.emit()
        else:
            print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if dog is not None:
        dog.cancel()


class _Watchdog:
    """Prints rank 0's result line exactly once — normally (emit), or from the timer with the probe marked as
    stalled — and on expiry ends the process (os._exit) so that no rank waits on a peer forever."""

    def __init__(self, res, rank: int, budget_s: float):
        import threading

        self.res, self.rank, self.budget_s = res, rank, budget_s
        self._lock = threading.Lock()
        self._printed = False
        self._timer = threading.Timer(budget_s, self._expire)
        self._timer.daemon = True
        self._timer.start()

    def emit(self) -> None:
        with self._lock:
            if not self._printed and self.rank == 0:
                print(json.dumps(self.res), flush=True)
            self._printed = True

    def _expire(self) -> None:
        with self._lock:
            if not self._printed and self.rank == 0:
                self.res["notes"].setdefault("xgpu_probe", {"error": f"no result within {self.budget_s:.0f} s"})
                print(json.dumps(self.res), flush=True)
            self._printed = True
        os._exit(0)

    def cancel(self) -> None:
        self._timer.cancel()


if __name__ == "__main__":
    main()
