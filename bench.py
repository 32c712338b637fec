#!/usr/bin/env python3
"""
Headline benchmark (BASELINE.json): req/s + p50 end-to-end latency of
Llama-3-8B batched serving on 1/2/4/8 MI355X.

Each rank (one per GPU, under torch.distributed.run for N > 1) runs a full
serving replica — data parallel, the right layout for an 8B model that fits one
288 GB GPU many times over — and the whole serving path minus TCP:

    Batcher(max_batch=32, max_latency=10 ms)  →  AsyncLLMEngine (engine thread)
      → continuous-batching scheduler → paged-KV Llama-3-8B (random-init bf16)
      → hand-written gfx950 kernels + hipBLASLt GEMMs, hipGraph decode.

One "step" = one wave of ``--batch`` (32) synthetic requests per GPU, each a
distinct random 512-token prompt generating 128 tokens (ignore_eos), submitted
together and served to completion (prefill + 128 decode iterations, sampling
included). Weak scaling: per-GPU work is fixed as N grows. ``value`` is the
whole-job request rate over the ranks that actually ran (``notes.world_size_seen``,
``notes.devices``); ``p50_latency_ms`` is the median submit→finish latency over
every timed request.

``--gpus N`` (N > 1) without a launcher starts ``torch.distributed.run`` with N
ranks as a CHILD process and relays its result line and exit status; it never
counts replicas that did not run. Under a launcher, ``--gpus`` must equal
WORLD_SIZE.

After the timed region of a multi-GPU run (its engines freed) the node measures
BASELINE configs 3 and 4 and the links they use (``notes.cross_gpu``, status
also at the top level as ``cross_gpu_status``): cross-GPU transports
(src/parallel/xgpu_probe.py), 8B disaggregated serving with prefill on rank 2k
and decode on rank 2k+1 (N >= 2), and a Llama-3-70B TP=N engine serving one
wave (N == 8) (src/parallel/node_bench.py). That section runs in its OWN
torch.distributed.run (a child of rank 0, one rank per GPU again), so a crash,
GPU fault or hang there cannot cost the timed result: rank 0 waits at most
``--cross-gpu-budget-s``, kills the child's process group on expiry, prints the
result with ``cross_gpu_status: "stalled ..."`` and exits 3.

    python bench.py                      # 1 GPU, 3 timed steps, 1 warmup
    python bench.py --gpus 8 --steps 3   # spawns the 8-rank launcher itself
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 3 --warmup 1
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import signal
import socket
import statistics
import subprocess
import sys
import threading
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC_FMT = "req/sec + p50 end-to-end latency, {model} batched serving at 1/2/4/8 MI355X"
STALL_EXIT = 3


def model_label(preset: str) -> str:
    """Display name of a preset: llama3-8b -> Llama-3-8B, mixtral-8x7b -> Mixtral-8x7B."""
    from src.models.presets import get_preset

    name = getattr(get_preset(preset), "name", None) or preset
    if name.startswith("llama3"):
        name = "Llama-3" + name[len("llama3"):]
    elif name.startswith("mixtral"):
        name = "Mixtral" + name[len("mixtral"):]
    return name.replace("-8b", "-8B").replace("-70b", "-70B").replace("x7b", "x7B")


def parse(argv=None):
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
    p.add_argument("--no-gemm-table", action="store_true", help="prefill GEMMs on the library defaults (A/B)")
    p.add_argument("--no-gemm-residual", action="store_true",
                   help="prefill o / down written out and added by the norm pass instead of in the GEMM epilogue (A/B)")
    p.add_argument("--decode-window", type=int, default=None, help="decode steps per hipGraph window (engine default)")
    p.add_argument("--tp", type=int, default=1, help="tensor-parallel degree per replica (70B: --tp 8)")
    p.add_argument("--moe-parallel", choices=["tp", "ep"], default="tp", help="MoE layout under --tp")
    p.add_argument("--sequence-parallel", action="store_true", help="Megatron-SP prefill under --tp")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: reference-op engine over gloo (tests the multi-rank plumbing, not a measurement)")
    p.add_argument("--decode-weights", default="auto", choices=("auto", "tiled", "single"),
                   help="EngineConfig.decode_weight_layout (A/B: single = decode on the row-major weights)")
    p.add_argument("--kv-blocks", type=int, default=None,
                   help="KV pool blocks per replica (default: the HBM left after the weights; --same-device: enough "
                        "for one wave, so the ranks sharing the GPU do not each claim its HBM)")
    p.add_argument("--same-device", action="store_true",
                   help="rehearsal: every rank on cuda:0, gloo coordinates (no RCCL; numbers are not a scaling point)")
    # the post-timed-region node section (configs 3 / 4 and the cross-GPU transports)
    p.add_argument("--cross-gpu", choices=["auto", "on", "off"], default="auto",
                   help="auto: on for multi-rank GPU runs; on: also on CPU (plumbing tests)")
    p.add_argument("--cross-gpu-budget-s", type=float, default=720.0, help="watchdog for the whole node section")
    p.add_argument("--disagg-preset", default=None, help="config 3 model (default: --preset)")
    p.add_argument("--tp-wave-preset", default="llama3-70b", help="config 4 model")
    p.add_argument("--tp-wave-min-world", type=int, default=8, help="run the config-4 TP wave from this many ranks")
    p.add_argument("--lb-preset", default="mixtral-8x7b", help="config 5 model (one worker per rank)")
    p.add_argument("--lb-kv-blocks", type=int, default=2048, help="config 5: KV blocks per worker (below the working set)")
    p.add_argument("--lb-requests-per-worker", type=int, default=32)
    p.add_argument("--no-lb-serving", action="store_true", help="skip the config-5 part of the node section")
    p.add_argument("--node-section-only", action="store_true",
                   help="internal: the node section alone (the child run that rank 0 of a multi-rank run starts)")
    p.add_argument("--verbose", action="store_true")
    return p.parse_args(argv)


# ------------------------------------------------------------------------------------------------ launch guard
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def needs_launcher(args) -> bool:
    """--gpus N > 1 outside torch.distributed.run: this process would be ONE replica."""
    return bool(args.gpus and args.gpus > 1 and "WORLD_SIZE" not in os.environ)


def self_launch(args, argv) -> int:
    """Run this script under torch.distributed.run with ``args.gpus`` ranks as a child process (no exec: this
    process has not touched the GPU and never will), relay rank 0's single JSON line to stdout and return the
    launcher's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    for ln in p.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if len(lines) != 1:
        print(f"bench.py: the {args.gpus}-rank run printed {len(lines)} result lines (rc {p.returncode})",
              file=sys.stderr)
        return p.returncode or 1
    print(lines[0], flush=True)
    return p.returncode


# ------------------------------------------------------------------------------------------------ serving
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


def serve_timed(args, rank, world, dev, on_gpu):
    """Build this rank's replica (or TP group member), run warmup + timed waves, return the measurements.
    Every engine object is local to this function, so its HBM is released when it returns."""
    from src.batcher import Batcher
    from src.config import EngineConfig
    from src.engine import LLMEngine
    from src.engine.async_engine import AsyncLLMEngine
    from src.preproc import normalize_request
    from src.utils.tracing import prof_marker

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)

    kv_blocks = args.kv_blocks
    if kv_blocks is None and args.same_device:
        kv_blocks = args.batch * -(-args.max_model_len // 16) + 64
    cfg = EngineConfig(max_num_seqs=args.batch, max_num_batched_tokens=max(16384, args.prompt_len),
                       num_kv_blocks=kv_blocks, max_latency_ms=args.max_latency_ms, use_cuda_graph=not args.no_graph,
                       graph_batch_sizes=[1, 2, 4, 8, 16, 24, 32, args.batch],
                       async_decode=not args.no_async_decode, tuned_gemm_table=not args.no_gemm_table,
                       decode_weight_layout=args.decode_weights,
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
            return {"elapsed": 0.0, "lats": [], "follower": True}
        engine = obj
    else:
        engine = LLMEngine.from_preset(args.preset, device=dev, cfg=cfg, max_model_len=args.max_model_len,
                                       seed=1234, capture=not args.no_graph)
        if args.no_gemm_residual:
            engine.model.prefill_gemm_residual = False
    engine.eos_token_id = None
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
        for _ in range(args.warmup):
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
    return {"elapsed": elapsed, "lats": lats, "init_s": init_s,
            "gen_tok": st["generated_tokens"] - stats0["generated_tokens"],
            "prefill_s": st["prefill_time"] - stats0["prefill_time"],
            "decode_s": st["decode_time"] - stats0["decode_time"]}


# ------------------------------------------------------------------------------------------------ node section
def cross_gpu_section(args, rank, world, dev, on_gpu, state, progress: bool = False) -> dict:
    """Configs 3 / 4 and the transports, after the timed region. Every rank runs every part in the same order;
    ``state["part"]`` names the running part. progress (the child run's rank 0): one stdout line as each part
    starts and ends, so the parent knows what finished if the run dies or stalls."""
    from src.parallel.node_bench import NodeBenchArgs, disagg_part, free_device_memory, lb_serving_part, tp_wave_part

    free_device_memory()  # the timed replicas' weights, KV pools and graphs
    cpu = dist.new_group(list(range(world)), backend="gloo") if dist.get_backend() != "gloo" else None
    out: dict = {}
    nb = NodeBenchArgs(preset=args.disagg_preset or args.preset, tp_preset=args.tp_wave_preset, batch=args.batch,
                       prompt_len=args.prompt_len, gen_len=args.gen_len, max_model_len=args.max_model_len,
                       max_latency_ms=args.max_latency_ms, graphs=not args.no_graph, lb_preset=args.lb_preset,
                       lb_kv_blocks=args.lb_kv_blocks, lb_requests_per_worker=args.lb_requests_per_worker)
    parts = []
    if on_gpu:
        parts.append("xgpu_probe")
    parts.append("disagg")
    if not args.no_lb_serving:
        parts.append("lb_serving")
    if world >= args.tp_wave_min_world:
        parts.append("tp_wave")
    for part in parts:
        state["part"] = part
        if progress:
            print(json.dumps({"node_part_start": part}), flush=True)
        if args.verbose:
            print(f"[rank {rank}] node section: {part}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        try:
            if part == "xgpu_probe":
                from src.parallel.xgpu_probe import xgpu_probe

                r = xgpu_probe(rank, world, dev, rccl=not args.same_device)
            elif part == "disagg":
                r = disagg_part(nb, rank, world, dev, cpu)
            elif part == "lb_serving":
                r = lb_serving_part(nb, rank, world, dev, cpu)
            else:
                r = tp_wave_part(nb, rank, world, dev)
        except Exception as e:  # noqa: BLE001 — reported; the timed result stands on its own
            r = {"error": f"{type(e).__name__}: {e}"[:300]}
        if isinstance(r, dict):
            r.setdefault("part_s", round(time.perf_counter() - t0, 1))
        out[part] = r
        state.setdefault("done", {})[part] = r
        if progress:
            print(json.dumps({"node_part": part, "result": r}, default=str), flush=True)
        free_device_memory()
        dist.barrier(group=cpu)
    state["part"] = None
    return out


_LAUNCHER_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                  "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def run_node_child(args, argv, world: int, state: dict):
    """Rank 0: the node section in its own torch.distributed.run with ``world`` ranks (``--node-section-only``;
    no exec — a child process group). Returns (cross, stalled): the section's results as its rank 0 reported
    them — every finished part even when the run dies or is killed at the budget — with ``status`` 0 (all parts
    ok), 1 (a part failed or the run exited non-zero) or STALL_EXIT (killed at the budget; ``stalled_part``)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += list(argv) + ["--node-section-only"]
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCHER_VARS and not k.startswith("TORCHELASTIC_")}
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, start_new_session=True)
    stalled = False
    try:
        out, _ = p.communicate(timeout=args.cross_gpu_budget_s)
    except subprocess.TimeoutExpired:
        stalled = True
        try:
            os.killpg(p.pid, signal.SIGKILL)  # the launcher and every rank it started
        except ProcessLookupError:
            pass
        out, _ = p.communicate()
    done, final, started = {}, None, None
    for ln in (out or "").splitlines():
        d = None
        if ln.startswith("{"):
            try:
                d = json.loads(ln)
            except ValueError:
                d = None
        if not isinstance(d, dict):
            print(ln, file=sys.stderr)
        elif "node_part_start" in d:
            started = state["part"] = d["node_part_start"]
        elif "node_part" in d:
            done[d["node_part"]] = d["result"]
            state.setdefault("done", {})[d["node_part"]] = d["result"]
            started = state["part"] = None
        elif "node_section" in d:
            final = d["node_section"]
    if final is not None and not stalled and p.returncode == 0:
        errs = _part_errors(final)
        final["status"] = 1 if errs else 0
        return final, False
    cross = dict(done)
    if stalled:
        cross.update(status=STALL_EXIT, stalled_part=started)
    else:
        cross.update(status=1, error=f"node section run exited {p.returncode}"
                     + (f" in {started}" if started else ""), failed_part=started)
    return cross, stalled


def _part_errors(cross: dict) -> list:
    errs = []
    for name, r in cross.items():
        if not isinstance(r, dict):
            continue
        if r.get("error"):
            errs.append(name)
        elif name == "xgpu_probe" and any(isinstance(v, dict) and v.get("error") for v in r.values()):
            errs.append(name)
    return errs


class _Watchdog:
    """Prints rank 0's result line exactly once — normally (emit), or from the timer with the node section marked
    as stalled — and on expiry ends the process with status STALL_EXIT (3), so a stall can never look like a
    successful run."""

    def __init__(self, res, rank: int, budget_s: float, state=None):
        self.res, self.rank, self.budget_s = res, rank, budget_s
        self.state = state if state is not None else {}
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
                part = self.state.get("part")
                msg = f"stalled in {part or 'teardown'}: no result within {self.budget_s:.0f} s"
                self.res["cross_gpu_status"] = msg
                cross = self.res.setdefault("notes", {}).setdefault("cross_gpu", {})
                cross["status"] = STALL_EXIT
                cross["stalled_part"] = part
                # the parts that finished before the stall (state["done"], written by rank 0 as it goes)
                for k, v in (self.state.get("done") or {}).items():
                    cross.setdefault(k, v)
                print(json.dumps(self.res), flush=True)
            self._printed = True
        os._exit(STALL_EXIT)

    def cancel(self) -> None:
        self._timer.cancel()


# ------------------------------------------------------------------------------------------------ main
def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if needs_launcher(args):
        return self_launch(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report replicas that do not run",
              file=sys.stderr)
        return 2
    n_gpus = world
    on_gpu = args.device == "cuda"
    if world > 1:
        if on_gpu:
            torch.cuda.set_device(0 if args.same_device else local)
        dist.init_process_group("nccl" if on_gpu and not args.same_device else "gloo")  # nccl = RCCL over xGMI
    dev = torch.device(f"cuda:{0 if args.same_device else local}" if on_gpu else "cpu")
    if args.node_section_only:  # the child run of a multi-rank bench (run_node_child)
        cross = cross_gpu_section(args, rank, world, dev, on_gpu, {"part": None, "done": {}}, progress=rank == 0)
        if rank == 0:
            print(json.dumps({"node_section": cross}, default=str), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0

    from src.parallel.node_bench import device_identity, distinct_devices, free_device_memory

    m = serve_timed(args, rank, world, dev, on_gpu)
    elapsed, lats = m["elapsed"], m["lats"]
    ident = device_identity(dev)
    rank_elapsed = [elapsed]
    idents = [ident]
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rank_elapsed = [None] * world
        dist.all_gather_object(rank_elapsed, elapsed)
        elapsed = float(t.item())
        gathered = [None] * world
        dist.all_gather_object(gathered, lats)
        lats = [x for g in gathered for x in g]
        idents = [None] * world
        dist.all_gather_object(idents, ident)
    tp = args.tp if args.tp > 1 else None
    replicas = world // args.tp
    total_req = args.steps * args.batch * replicas
    res = None
    if rank == 0:
        label = model_label(args.preset)
        res = {
            "metric": METRIC_FMT.format(model=label),
            "value": round(total_req / elapsed, 3),
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
            "output_tok_per_s": round(m["gen_tok"] * replicas / elapsed, 1),
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
                "prefill_gemm_table": not args.no_gemm_table,
                "prefill_gemm_residual": not args.no_gemm_residual,
            },
            "notes": {
                "baseline": "reference publishes no numbers and has no GPU path (BASELINE.md); vs_baseline=null",
                "rank0_prefill_s": round(m["prefill_s"], 3),
                "rank0_decode_s": round(m["decode_s"], 3),
                "engine_init_s": round(m["init_s"], 1),
                "world_size_seen": dist.get_world_size() if world > 1 else 1,
                "distinct_devices": distinct_devices(idents),
                "devices": idents,
            },
        }
        if args.same_device:
            res["notes"]["rehearsal"] = "every rank on cuda:0: not a scaling point"
        if world > 1 and tp is None:  # the value uses the slowest replica; the spread shows stragglers
            res["notes"]["rank_elapsed_s"] = [round(x, 3) for x in rank_elapsed]
    m = None
    run_node = world > 1 and tp is None and (args.cross_gpu == "on" or (args.cross_gpu == "auto" and on_gpu))
    dog = None
    rc = 0
    cpu = None
    if run_node:
        state: dict = {"part": None, "done": {}}
        # outer guard: the child run is bounded by the budget; this covers this process's own teardown
        dog = _Watchdog(res, rank, args.cross_gpu_budget_s + 180.0, state)
        free_device_memory()  # the timed replicas' weights, KV pools and graphs, before the child takes the GPUs
        if dist.get_backend() != "gloo":
            import datetime

            cpu = dist.new_group(list(range(world)), backend="gloo",
                                 timeout=datetime.timedelta(seconds=args.cross_gpu_budget_s + 600))
        dist.barrier(group=cpu)
        if rank == 0:
            cross, stalled = run_node_child(args, argv, world, state)
            res["notes"]["cross_gpu"] = cross
            if stalled:
                res["cross_gpu_status"] = (f"stalled in {cross.get('stalled_part') or 'teardown'}: no result within "
                                           f"{args.cross_gpu_budget_s:.0f} s")
                rc = STALL_EXIT
            elif cross["status"]:
                errs = _part_errors(cross) or [cross.get("failed_part") or "the node section run"]
                res["cross_gpu_status"] = "error in " + ", ".join(errs)
            else:
                res["cross_gpu_status"] = "ok"
        dist.barrier(group=cpu)  # the other ranks wait here (CPU) while rank 0's child run has the GPUs
    if rank == 0:
        if dog is not None:
            dog.emit()
        else:
            print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier(group=cpu)
        dist.destroy_process_group()
    if dog is not None:
        dog.cancel()
    return rc


if __name__ == "__main__":
    sys.exit(main())
