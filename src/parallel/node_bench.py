"""
BASELINE configs 3 and 4 measured by a multi-GPU ``bench.py`` run on the node itself, after its timed
data-parallel region (and after that region's engines are freed):

* :func:`disagg_part` (config 3, N >= 2): Llama-3-8B disaggregated serving. Rank 2k is a prefill worker,
  rank 2k+1 a decode worker (:class:`src.worker.Worker` + :class:`src.engine.backend.LLMBackend`, the
  production classes): each prompt's KV is gathered by the prefill GPU straight into the decode GPU's IPC
  landing zone (shader stores over xGMI), only metadata crosses the RPC socket, and the decode engine joins
  the sequence to its continuous batch. One wave of ``batch`` x (prompt -> gen) requests per pair, timed;
  req/s, p50 latency, TTFT and how the KV travelled (``kv_path``; anything but ``direct`` on a GPU node is
  reported as a failure).
* :func:`lb_serving_part` (config 5, N >= 2): Mixtral-8x7B, one worker per GPU (the production Worker +
  LLMBackend) behind ONE coordinator on rank 0 whose load balancer picks a worker per request
  (``least_latency`` on the workers' engine reports, then ``round_robin`` for comparison), config 5's
  mixed-length workload with Zipf-shared prefixes and KV pools smaller than its working set (LRU / TTL
  evictions): req/s, p50 / p99, TTFT, dispatches per worker, prefix hits, evictions
  (:mod:`src.parallel.lb_serving`).
* :func:`tp_wave_part` (config 4, N == 8 by default): Llama-3-70B tensor-parallel over every rank — Megatron
  split, one-shot IPC exchange fused into the row-parallel GEMM epilogue, RCCL for prefill-sized
  all-reduces — one wave served to completion: ms per decode step, req/s of the TP group, whether the fused
  exchange ran, and the group's error word.

Both run every collective in the same order on every rank whatever fails locally; a local failure is
returned as an ``error`` string. The caller (bench.py) bounds the whole section with a watchdog.

Reference: the reference names these configurations but has no GPU path (`/root/reference/README.md:15`,
`/root/reference/src/router.py:140-184`, `/root/reference/src/model_registry.py:149-161`).
"""

from __future__ import annotations

import asyncio
import gc
import os
import random
import statistics
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist


@dataclass
class NodeBenchArgs:
    preset: str = "llama3-8b"            # config 3 model
    tp_preset: str = "llama3-70b"        # config 4 model
    batch: int = 32
    prompt_len: int = 512
    gen_len: int = 128
    max_model_len: int = 2048
    max_latency_ms: float = 10.0
    warmup: int = 1                      # untimed waves before the timed one(s)
    waves: int = 1
    kv_blocks: int = 8192                # per engine (these parts never need the whole HBM)
    graphs: bool = True
    lb_preset: str = "mixtral-8x7b"      # config 5 model
    lb_kv_blocks: int = 2048             # per worker: below the shared-prefix working set, so the pools evict
    lb_requests_per_worker: int = 32
    lb_strategies: tuple = ("least_latency", "round_robin")


def device_identity(dev: torch.device) -> Dict[str, Any]:
    """What this rank runs on, for the proof-of-ranks record (UUID / PCI ids where the runtime reports them)."""
    out: Dict[str, Any] = {"pid": os.getpid(), "host": os.uname().nodename}
    if dev.type != "cuda":
        out["device"] = "cpu"
        return out
    p = torch.cuda.get_device_properties(dev)
    out["device"] = str(dev)
    out["name"] = p.name
    for k in ("uuid", "pci_bus_id", "pci_device_id", "pci_domain_id"):
        v = getattr(p, k, None)
        if v is not None:
            out[k] = str(v)
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if os.environ.get(k):
            out[k] = os.environ[k]
    return out


def distinct_devices(ids: List[Dict[str, Any]]) -> int:
    """Distinct physical devices among the ranks' identities (host + UUID, else host + PCI location)."""
    keys = set()
    for d in ids:
        if d.get("device") == "cpu":
            keys.add((d.get("host"), "cpu", d.get("pid")))
        else:
            keys.add((d.get("host"), d.get("uuid") or (d.get("pci_domain_id"), d.get("pci_bus_id"),
                                                         d.get("pci_device_id")) or d.get("device")))
    return len(keys)


def free_device_memory() -> None:
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def _prompts(rng: random.Random, n: int, length: int, vocab: int) -> List[List[int]]:
    return [[rng.randrange(3, vocab) for _ in range(length)] for _ in range(n)]


def _arch_of(preset: str) -> str:
    return "mixtral" if preset.startswith("mixtral") else "llama"


# ------------------------------------------------------------------------------------------------ config 3
def disagg_part(a: NodeBenchArgs, rank: int, world: int, dev: torch.device, cpu_group) -> Dict[str, Any]:
    """Every rank calls this. Returns rank 0's aggregate (other ranks: their own record)."""
    return asyncio.run(_disagg(a, rank, world, dev, cpu_group))


async def _disagg(a: NodeBenchArgs, rank: int, world: int, dev: torch.device, cpu_group) -> Dict[str, Any]:
    from src.config import ModelConfig
    from src.engine.backend import LLMBackend
    from src.worker import Worker

    loop = asyncio.get_running_loop()
    pairs = world // 2
    role = None if rank >= 2 * pairs else ("prefill" if rank % 2 == 0 else "decode")

    def mcfg(r: str, extra: Dict[str, Any]) -> ModelConfig:
        return ModelConfig(model_name="llama", model_path="", max_batch_size=a.batch, arch=_arch_of(a.preset),
                           preset=a.preset, role=r, max_model_len=a.max_model_len, max_latency_ms=a.max_latency_ms,
                           use_cuda_graph=a.graphs, num_kv_blocks=a.kv_blocks, seed=1234,
                           overrides=dict(device=str(dev), **extra))

    async def coll(fn):  # a blocking host collective, off the event loop (a decode worker keeps serving)
        return await loop.run_in_executor(None, fn)

    worker = backend = None
    rec: Dict[str, Any] = {"rank": rank, "role": role, "device": str(dev)}
    try:
        if role == "decode":
            worker = Worker(f"decode-r{rank}", host="127.0.0.1", port=0, install_signal_handlers=False)
            if not worker.load_model(mcfg("decode", {})):
                raise RuntimeError("decode model failed to load")
            await worker.start()
    except Exception as e:  # noqa: BLE001 — reported through the gather below
        rec["error"] = f"decode worker: {e}"[:300]
        worker = None
    addrs: List[Optional[str]] = [None] * world
    mine = worker.address if worker is not None else None
    await coll(lambda: dist.all_gather_object(addrs, mine, group=cpu_group))
    try:
        if role == "prefill":
            peer = addrs[rank + 1]
            if peer is None:
                raise RuntimeError(f"no decode worker on rank {rank + 1}")
            backend = LLMBackend(mcfg("prefill", {"decode_worker": peer}))
            await backend.start()
            rec.update(await _disagg_waves(backend, a, rank))
    except Exception as e:  # noqa: BLE001
        rec["error"] = f"{type(e).__name__}: {e}"[:300]
    await coll(lambda: dist.barrier(group=cpu_group))  # decode workers serve until every prefill rank is done
    if worker is not None:
        try:
            st = await worker.handle_message({"op": "engine_stats", "model": "llama"})
            rec["kv_zone"] = (st.get("stats") or {}).get("kv_zone")
        except Exception:  # noqa: BLE001
            pass
    recs: List[Any] = [None] * world
    await coll(lambda: dist.all_gather_object(recs, rec, group=cpu_group))
    for obj in (backend, worker):
        try:
            if obj is backend and obj is not None:
                await obj.stop()
                obj.close()
            elif obj is not None:
                await obj.shutdown()
        except Exception:  # noqa: BLE001
            pass
    backend = worker = None
    free_device_memory()
    if rank != 0:
        return rec
    return _disagg_summary(recs, a, dev)


async def _disagg_waves(backend, a: NodeBenchArgs, rank: int) -> Dict[str, Any]:
    rng = random.Random(7000 + rank)
    vocab = backend.engine.arch.vocab_size
    backend.engine.eos_token_id = None

    async def wave(prompts):
        async def one(p):
            t0 = time.perf_counter()
            out = await backend.predict({"prompt_token_ids": p, "max_tokens": a.gen_len, "ignore_eos": True,
                                         "return_text": False})
            if out.get("num_output_tokens") != a.gen_len or not out.get("disaggregated"):
                raise RuntimeError(f"bad disaggregated reply: {dict((k, out.get(k)) for k in ('num_output_tokens', 'disaggregated', 'finish_reason'))}")
            return time.perf_counter() - t0, out.get("ttft_ms")

        return await asyncio.gather(*(one(p) for p in prompts))

    for _ in range(a.warmup):
        await wave(_prompts(rng, a.batch, a.prompt_len, vocab))

    async def timed() -> Dict[str, Any]:
        waves = [_prompts(rng, a.batch, a.prompt_len, vocab) for _ in range(a.waves)]
        if backend.engine.device.type == "cuda":
            torch.cuda.synchronize(backend.engine.device)
        t0 = time.perf_counter()
        res: List[Any] = []
        for w in waves:
            res += await wave(w)
        el = time.perf_counter() - t0
        lat = sorted(x[0] * 1e3 for x in res)
        ttft = sorted(x[1] for x in res if x[1] is not None)
        return {"requests": len(res), "elapsed_s": round(el, 4), "req_s": round(len(res) / el, 3),
                "p50_latency_ms": round(statistics.median(lat), 2),
                "ttft_p50_ms": round(statistics.median(ttft), 2) if ttft else None,
                "ttft_p99_ms": round(ttft[max(0, int(0.99 * len(ttft)) - 1)], 2) if ttft else None}

    link = backend._decode_link
    out = await timed()
    st = link.stats() if link is not None else {}
    out.update(kv_path=st.get("kv_path"), kv_link=st)
    # transport A/B on the same pair: the default has the prefill GPU's gather kernel store straight into
    # the decode GPU's landing zone over xGMI (CUs do the transfer, beside the next prefill's GEMMs); the alternative
    # gathers locally and lets the copy engines move the packet (hipMemcpyAsync peer copy, CUs left to the GEMMs)
    ch = getattr(link, "_ipc", None) if link is not None else None
    if ch is not None and backend.engine.device.type == "cuda":
        kv_direct0 = backend.kv_direct
        try:
            backend.kv_direct, ch.dma = False, True
            n0 = link.staged_packets
            alt = await timed()
            alt["staged_packets"] = link.staged_packets - n0
            out["transport_ab"] = {"shader_stores_direct": {k: out[k] for k in ("req_s", "p50_latency_ms",
                                                                               "ttft_p50_ms", "ttft_p99_ms")},
                                   "copy_engine_staged": alt}
        except Exception as e:  # noqa: BLE001 — the A/B must not cost the default result
            out["transport_ab"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        finally:
            backend.kv_direct, ch.dma = kv_direct0, False
    return out


def _disagg_summary(recs: List[Dict[str, Any]], a: NodeBenchArgs, dev: torch.device) -> Dict[str, Any]:
    pre = [r for r in recs if r and r.get("role") == "prefill"]
    errors = {r["rank"]: r["error"] for r in recs if r and r.get("error")}
    ok = [r for r in pre if "req_s" in r]
    out: Dict[str, Any] = {
        "config": "BASELINE 3: prefill worker on rank 2k -> decode worker on rank 2k+1, KV into the decode GPU's "
                  "IPC landing zone",
        "model": a.preset, "pairs": len(pre), "batch_per_pair": a.batch, "prompt_len": a.prompt_len,
        "gen_len": a.gen_len, "timed_waves": a.waves,
        "per_pair": [{k: r.get(k) for k in ("rank", "req_s", "p50_latency_ms", "ttft_p50_ms", "ttft_p99_ms",
                                            "kv_path", "transport_ab")} for r in pre],
        "decode_zones": [r.get("kv_zone") for r in recs if r and r.get("role") == "decode"],
    }
    if ok:
        out["req_s_total"] = round(sum(r["req_s"] for r in ok), 3)
        out["p50_latency_ms"] = round(statistics.median(r["p50_latency_ms"] for r in ok), 2)
        ttfts = [r["ttft_p50_ms"] for r in ok if r.get("ttft_p50_ms") is not None]
        out["ttft_p50_ms"] = round(statistics.median(ttfts), 2) if ttfts else None
        out["kv_path"] = "+".join(sorted({str(r.get("kv_path")) for r in ok}))
    # on GPUs the KV must never ride the socket: a byte-path packet is a failed configuration
    if dev.type == "cuda":
        for r in ok:
            if r.get("kv_path") != "direct":
                errors.setdefault(r["rank"], f"kv_path {r.get('kv_path')!r}: the KV did not go GPU to GPU directly")
    if errors or len(ok) != len(pre) or not pre:
        out["error"] = errors or "no prefill pair completed"
    return out


# ------------------------------------------------------------------------------------------------ config 5
def lb_serving_part(a: NodeBenchArgs, rank: int, world: int, dev: torch.device, cpu_group) -> Dict[str, Any]:
    """Every rank calls this. Returns rank 0's aggregate (other ranks: their own record)."""
    return asyncio.run(_lb_serving(a, rank, world, dev, cpu_group))


async def _lb_serving(a: NodeBenchArgs, rank: int, world: int, dev: torch.device, cpu_group) -> Dict[str, Any]:
    from src.config import ModelConfig
    from src.parallel.lb_serving import LBWorkload, make_requests, serve_through_coordinator
    from src.worker import Worker

    loop = asyncio.get_running_loop()

    async def coll(fn):
        return await loop.run_in_executor(None, fn)

    arch = _arch_of(a.lb_preset)
    rec: Dict[str, Any] = {"rank": rank}
    worker = None
    t0 = time.perf_counter()
    try:
        worker = Worker(f"lb-r{rank}", host="127.0.0.1", port=0, install_signal_handlers=False)
        cfg = ModelConfig(model_name="moe", model_path="", max_batch_size=a.batch, arch=arch, preset=a.lb_preset,
                          max_model_len=a.max_model_len + 256, max_latency_ms=a.max_latency_ms,
                          use_cuda_graph=a.graphs, num_kv_blocks=a.lb_kv_blocks, seed=1234,
                          overrides={"device": str(dev), "kv_block_ttl_s": 30.0})
        if not worker.load_model(cfg):
            raise RuntimeError("worker model failed to load")
        await worker.start()
        rec["init_s"] = round(time.perf_counter() - t0, 1)
    except Exception as e:  # noqa: BLE001 — reported through the gather below
        rec["error"] = f"worker: {type(e).__name__}: {e}"[:300]
        worker = None
    addrs: List[Any] = [None] * world
    mine = (worker.worker_id, worker.address) if worker is not None else None
    await coll(lambda: dist.all_gather_object(addrs, mine, group=cpu_group))
    runs: List[Dict[str, Any]] = []
    if rank == 0:
        try:
            workers = {w: ad for w, ad in (x for x in addrs if x is not None)}
            if len(workers) != world:
                raise RuntimeError(f"only {len(workers)} of {world} workers came up")
            vocab = worker.models["moe"].engine.arch.vocab_size
            n = a.lb_requests_per_worker * world
            for i, strat in enumerate(a.lb_strategies):
                # a fresh prefix set per strategy (the previous run's cached prefixes must not favour the next)
                # config 5's mix (128-2048 -> 32-256) at serving sizes; scaled down for small test contexts
                big = a.max_model_len >= 1024
                pmax = min(2048, a.max_model_len)
                shape = dict(prompt_min=min(128, pmax // 2), prompt_max=pmax,
                             gen_choices=(32, 64, 128, 256) if big else (4, 8, 16))
                wl = LBWorkload(requests=n, concurrency=min(n, 8 * world), seed=100 + i, **shape)
                warm = make_requests(LBWorkload(requests=2 * world, seed=900 + i, **shape), vocab)
                runs.append(await serve_through_coordinator(workers, "moe", arch, strat, make_requests(wl, vocab),
                                                            wl.concurrency, warmup=warm))
        except Exception as e:  # noqa: BLE001
            rec["error"] = f"{type(e).__name__}: {e}"[:300]
    await coll(lambda: dist.barrier(group=cpu_group))  # every worker serves until rank 0's runs are done
    if worker is not None:
        try:
            await worker.shutdown()
        except Exception:  # noqa: BLE001
            pass
    worker = None
    free_device_memory()
    recs: List[Any] = [None] * world
    await coll(lambda: dist.all_gather_object(recs, rec, group=cpu_group))
    if rank != 0:
        return rec
    errors = {r["rank"]: r["error"] for r in recs if r and r.get("error")}
    out: Dict[str, Any] = {
        "config": "BASELINE 5: one worker per GPU behind one coordinator; the load balancer picks per request",
        "model": a.lb_preset, "workers": world, "kv_blocks_per_worker": a.lb_kv_blocks,
        "workload": "mixed 128-2048 -> 32-256 tokens, Zipf-shared prefixes, closed loop",
        "runs": runs, "worker_init_s": [r.get("init_s") for r in recs if r],
    }
    ll = next((r for r in runs if r.get("strategy") == "least_latency"), None)
    if ll is not None:
        out.update({k: ll.get(k) for k in ("req_s", "p50_latency_ms", "p99_latency_ms", "ttft_p50_ms",
                                           "prefix_hit_rate", "lru_evictions", "ttl_evictions")})
        out["dispatched_per_worker"] = {w: p["dispatched"] for w, p in ll["per_worker"].items()}
    if any(r.get("error_count") for r in runs):
        errors.setdefault(0, f"request errors: {[r.get('errors') for r in runs]}"[:300])
    if errors or not runs:
        out["error"] = errors or "no run completed"
    return out


# ------------------------------------------------------------------------------------------------ config 4
def tp_wave_part(a: NodeBenchArgs, rank: int, world: int, dev: torch.device) -> Dict[str, Any]:
    """A TP=world engine of ``a.tp_preset`` over every rank; rank 0 (the leader) serves warm-up + timed waves
    of ``a.batch`` requests with ``generate`` while the followers mirror its steps. Every rank calls this."""
    from src.config import EngineConfig
    from src.parallel.tp import init_tp
    from src.parallel.tp_runner import build_tp_engine
    from src.preproc import SamplingParams

    t_init = time.perf_counter()
    tp = init_tp(world)
    cfg = EngineConfig(max_num_seqs=a.batch, max_num_batched_tokens=max(16384, a.prompt_len), num_kv_blocks=a.kv_blocks,
                       max_latency_ms=0.0, use_cuda_graph=a.graphs,
                       graph_batch_sizes=sorted({1, 2, 4, 8, 16, 24, 32, a.batch}))
    obj = build_tp_engine(a.tp_preset, tp, dev, cfg=cfg, max_model_len=a.max_model_len, seed=1234, capture=a.graphs)
    init_s = time.perf_counter() - t_init
    res: Dict[str, Any] = {"rank": rank}
    try:
        if rank != 0:
            obj.follower_loop()
            return res
        eng = obj
        eng.eos_token_id = None
        rng = random.Random(99)
        vocab = eng.arch.vocab_size
        sp = SamplingParams(max_tokens=a.gen_len, ignore_eos=True)
        try:
            for _ in range(a.warmup):
                eng.generate(_prompts(rng, a.batch, a.prompt_len, vocab), sp)
            waves = [_prompts(rng, a.batch, a.prompt_len, vocab) for _ in range(a.waves)]
            st0 = dict(eng.stats)
            t0 = time.perf_counter()
            outs: List[List[int]] = []
            for w in waves:
                outs += eng.generate(w, sp)
            el = time.perf_counter() - t0
            st = eng.stats
            # decode steps, not engine iterations: every request's first token comes from its prefill, the
            # other gen_len - 1 from decode steps (an engine iteration is a whole window of them)
            steps = max(1, (a.gen_len - 1) * a.waves)
            dec = st["decode_time"] - st0["decode_time"]
            car = tp.car
            res.update({
                "config": "BASELINE 4: tensor-parallel engine over every rank of the node",
                "model": a.tp_preset, "tp": world, "batch": a.batch, "prompt_len": a.prompt_len, "gen_len": a.gen_len,
                "timed_waves": a.waves, "requests": len(outs),
                "all_tokens": all(len(o) == a.gen_len for o in outs),
                "req_s": round(len(outs) / el, 3), "ms_per_wave": round(1e3 * el / a.waves, 2),
                "decode_ms_per_step": round(1e3 * dec / steps, 3),
                "prefill_ms_per_wave": round(1e3 * (st["prefill_time"] - st0["prefill_time"]) / a.waves, 2),
                "fused_exchange": bool(eng.model.decode_plan(a.batch).get("tp_fused")),
                # the group's measured choice between the fused and the separate exchange (engine build)
                "exchange_calibration": getattr(eng.model, "tp_exchange_calibration", None),
                "one_shot_ipc": car is not None,
                "error_word": bool(car.error()) if car is not None else None,
                "graphs_replayed": bool(eng.runner.graphs),
                "decode_windows": st.get("decode_windows", 0) - st0.get("decode_windows", 0),
                "queued_windows": st.get("queued_windows", 0) - st0.get("queued_windows", 0),
                "windows_mirrored": getattr(eng.runner, "windows_synced", 0),
                "rank_weight_gib": round(eng.model.weight_bytes() / 2**30, 2),
                "engine_init_s": round(init_s, 1),
            })
            if not res["all_tokens"]:
                res["error"] = "a request did not produce gen_len tokens"
        finally:
            eng.runner.stop_followers()
        return res
    finally:
        if tp.car is not None:
            try:
                tp.car.close()
            except Exception:  # noqa: BLE001
                pass
            tp.car = None
        obj = None
        free_device_memory()
