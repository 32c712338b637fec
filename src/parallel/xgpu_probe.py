"""
Cross-GPU probe run by a multi-GPU ``bench.py`` after its timed region: the data movements the serving
configurations rely on, measured between real GPUs of the node (one process per GPU) instead of between
two processes sharing one GPU.

* ``rccl_allreduce``: RCCL (``torch.distributed`` backend "nccl") all-reduce of a 256 MiB bf16 tensor —
  algorithm and bus bandwidth (bus = 2 (n - 1) / n x bytes / time, the per-link figure a ring over xGMI is
  bound by).
* ``ipc_allreduce``: the one-shot IPC all-reduce of the tensor-parallel decode path
  (:class:`src.parallel.custom_allreduce.CustomAllReduce`, the protocol the fused row-parallel GEMM epilogue
  uses) at decode sizes (32 rows x 4,096 / 8,192 bf16): latency, and its sum checked against RCCL's.
* ``kv_hop``: the disaggregated prefill -> decode KV hand-off — rank 2k gathers a 128 MiB packet straight
  into rank 2k+1's IPC landing zone (:class:`IPCLandingZone` / :class:`IPCSender`, shader stores over
  xGMI), rank 2k+1 checks every byte; GB/s of the copy.

* ``tp_engine``: a TP=N engine (llama-mini) over all ranks — hipGraph decode windows with the exchange in the
  row-parallel GEMM epilogue over the links — whose greedy tokens are checked against a TP=1 recompute.

Everything is bounded: the caller runs this under a watchdog (bench.py), every device wait is an event
poll or a collective, and each part reports an error string instead of raising. Reference: the reference
has no GPU path; these are the transports behind its placement / disaggregation claims
(`/root/reference/README.md:14-15`, `/root/reference/src/router.py:140-184`).

Rehearsal with N ranks on ONE GPU (no RCCL: it refuses two ranks on one device; gloo coordinates)::

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \\
        -m src.parallel.xgpu_probe --same-device
"""

from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


def _events():
    return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def _rccl_allreduce(dev, world: int, group=None) -> Dict[str, Any]:
    n = 128 << 20  # 128 M bf16 = 256 MiB
    t = torch.ones(n, dtype=torch.bfloat16, device=dev)
    for _ in range(2):
        dist.all_reduce(t, group=group)
    torch.cuda.synchronize(dev)
    iters = 5
    e0, e1 = _events()
    dist.barrier(group=group)
    e0.record()
    for _ in range(iters):
        dist.all_reduce(t, group=group)
    e1.record()
    torch.cuda.synchronize(dev)
    s = e0.elapsed_time(e1) / 1e3 / iters
    nbytes = n * 2
    return {"bytes": nbytes, "ms": round(s * 1e3, 3), "algbw_GBps": round(nbytes / s / 1e9, 1),
            "busbw_GBps": round(2 * (world - 1) / world * nbytes / s / 1e9, 1)}


def _ipc_allreduce(rank: int, world: int, dev, group=None, rccl_group=None) -> Dict[str, Any]:
    from src.parallel.custom_allreduce import CustomAllReduce

    car = CustomAllReduce(rank, world, group=group)
    out: Dict[str, Any] = {}
    try:
        g = torch.Generator(device="cpu").manual_seed(17 + rank)
        for rows, hid in ((32, 4096), (32, 8192)):
            x = (torch.randn(rows, hid, generator=g) * 0.5).to(torch.bfloat16).to(dev)
            y = car.all_reduce(x)
            torch.cuda.synchronize(dev)
            ok = None
            if rccl_group is not False:  # the reference sum: RCCL over the same inputs (fp32 accumulate)
                ref = x.float()
                dist.all_reduce(ref, group=rccl_group)
                ok = bool(torch.allclose(y.float(), ref, rtol=2e-2, atol=2e-2))
            for _ in range(5):
                car.all_reduce(x, out=y)
            torch.cuda.synchronize(dev)
            iters = 50
            dist.barrier(group=group)
            e0, e1 = _events()
            e0.record()
            for _ in range(iters):
                car.all_reduce(x, out=y)
            e1.record()
            torch.cuda.synchronize(dev)
            out[f"{rows}x{hid}"] = {"bytes": rows * hid * 2, "us": round(e0.elapsed_time(e1) * 1e3 / iters, 2),
                                    "matches_rccl": ok}
        out["fused_row_parallel"] = _fused_row_parallel(rank, world, dev, car, group, rccl_group)
        out["error_word"] = bool(car.error())
    finally:
        dist.barrier(group=group)
        car.close()
    return out


def _timed(fn, dev, group, iters: int = 20) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize(dev)
    dist.barrier(group=group)
    e0, e1 = _events()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) * 1e3 / iters


def _fused_row_parallel(rank: int, world: int, dev, car, group=None, rccl_group=None) -> Dict[str, Any]:
    """The tensor-parallel decode layer's row-parallel projections at Llama-3-70B's shard shapes for this group
    size (o: K = 8,192 / world, down: K = 28,672 / world, N = 8,192, 32 rows): ONE launch whose column tiles'
    last arrivers exchange over the group (gemm_decode_car) against the same GEMM without the exchange
    (mode 3 on the local K shard) — the difference is what the one-shot exchange costs over the links."""
    from src import ops

    res: Dict[str, Any] = {}
    shapes = [("o", 8192 // world, 8192), ("down", 28672 // world, 8192)]
    if car.ranks_per_gpu > 1:  # a one-GPU rehearsal: a shape whose waiting tiles leave room for every rank's grid
        shapes = [("rehearsal", 1024, 2048)]
    for name, k, n in shapes:
        if k % 256:
            res[name] = {"skipped": f"K = {k}"}
            continue
        wr, kc, sk = ops.decode_tile(n, k, 3, 32)
        half = None
        for h in (False, True):  # the model's choice (CausalLM._tp_fused_tile): full LDS ring, else the half ring
            if car.fused_ok(n // wr, (n // wr) * sk, ops.gd_occupancy(3, wr, kc, sk, 32, h)):
                half = h
                break
        if half is None:
            res[name] = {"skipped": "fused_ok"}
            continue
        g = torch.Generator(device="cpu").manual_seed(5 + rank)
        x = (torch.randn(32, k, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        w = (torch.randn(n, k, generator=g) * 0.02).to(torch.bfloat16).to(dev)
        resid = torch.zeros(32, n, dtype=torch.bfloat16, device=dev)
        ssp = torch.zeros(n // wr, ops.SSP_LD, dtype=torch.float32, device=dev)
        cnt = torch.zeros(n // wr, dtype=torch.int32, device=dev)
        car.row_parallel_residual(x, w, resid, ssp, cnt, wr, kc, sk, tiled=False, half_ring=half)
        torch.cuda.synchronize(dev)
        ok = None
        if rccl_group is not False:
            ref = x.float() @ w.float().t()
            dist.all_reduce(ref, group=rccl_group)
            ok = bool(torch.allclose(resid.float(), ref, rtol=3e-2, atol=3e-2))
        fused = _timed(lambda: car.row_parallel_residual(x, w, resid, ssp, cnt, wr, kc, sk, tiled=False,
                                                         half_ring=half), dev, group)
        resid2 = torch.zeros_like(resid)
        ssp2, cnt2 = torch.zeros_like(ssp), torch.zeros_like(cnt)
        local = _timed(lambda: ops.linear_slab_residual(x, w, resid2, ssp2, cnt2, wr, sk, kc=kc, half_ring=half),
                       dev, group)
        # the same projection with the exchange as its own launch: bf16 partial GEMM, then the one-shot all-reduce +
        # residual + statistics kernel (what the engine runs when the residency rule refuses the fused form) ...
        ssp1 = torch.zeros(1, ops.SSP_LD, dtype=torch.float32, device=dev)
        sep = _timed(lambda: car.all_reduce_residual(ops.linear(x, w), resid2, ssp1), dev, group)
        row = {"K": k, "tile": [wr, kc, sk], "half_ring": half, "fused_us": round(fused, 2),
               "local_us": round(local, 2), "exchange_us": round(fused - local, 2),
               "separate_one_shot_us": round(sep, 2), "matches_rccl": ok}
        # ... and over RCCL (its ring / LL protocols over the xGMI links) for the same 32 x N message
        if rccl_group is not False:
            def rccl_path():
                part = ops.linear(x, w)
                dist.all_reduce(part, group=rccl_group)
                ops.residual_add_sumsq(resid2, part, ssp1)
            row["rccl_us"] = round(_timed(rccl_path, dev, group), 2)
        res[name] = row
    return res


def _kv_hop(rank: int, world: int, dev, group=None) -> Dict[str, Any]:
    """Every rank runs the same collectives in the same order whatever fails locally (a local error is
    recorded and reported through the final gather, never raised between two collectives)."""
    from src.parallel.kv_transfer import IPCLandingZone, IPCSender

    nbytes = 128 << 20
    recv = rank % 2 == 1
    paired = (rank ^ 1) < world
    res: Dict[str, Any] = {"bytes": nbytes, "pairs": world // 2}
    err: Optional[str] = None
    zone = sender = None
    info = None
    try:
        if recv and paired:
            zone = IPCLandingZone(dev, capacity=256 << 20, uncached=True)
            info = {"handle": zone.handle, "seg": zone.seg_bytes}
    except Exception as e:  # noqa: BLE001
        err = f"zone: {e}"[:200]
    allinfo: list = [None] * world
    dist.all_gather_object(allinfo, info, group=group)
    g = torch.Generator(device="cpu").manual_seed(99)
    payload = torch.randint(-30000, 30000, (nbytes // 2,), dtype=torch.int16, generator=g)
    try:
        if not recv and paired and allinfo[rank + 1] is not None:
            peer = allinfo[rank + 1]
            sender = IPCSender(peer["handle"], peer["seg"], dev)
            src = payload.to(dev).view(torch.bfloat16)
            sender.write(0, src).synchronize()  # warm the mapping
            e0, e1 = _events()
            e0.record(sender.stream)
            sender.write(0, src)
            e1.record(sender.stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            res["send_ms"] = round(ms, 3)
            res["GBps"] = round(nbytes / (ms / 1e3) / 1e9, 1)
    except Exception as e:  # noqa: BLE001
        err = f"send: {e}"[:200]
    dist.barrier(group=group)  # the sender's copy is complete before the receiver reads its zone
    match = None
    try:
        if zone is not None:
            match = bool(torch.equal(zone.views[0][:nbytes].view(torch.int16).cpu(), payload))
    except Exception as e:  # noqa: BLE001
        err = f"check: {e}"[:200]
    flags: list = [None] * world
    dist.all_gather_object(flags, {"GBps": res.get("GBps"), "receiver_bytes_match": match, "error": err},
                           group=group)
    res["per_rank"] = flags
    dist.barrier(group=group)
    for obj in (sender, zone):
        try:
            if obj is not None:
                obj.close()
        except Exception:  # noqa: BLE001
            pass
    return res


TP_PROMPTS = [[5, 9, 33, 12, 7] * 9, [100, 200, 300], list(range(3, 140))]


def _greedy_reference(model, prompt, n):
    """Greedy no-cache recompute on one GPU; also the top1-top2 logit margin per step."""
    from src.models.llama import AttnMetadata

    d = model.device
    ids, toks, margins = list(prompt), [], []
    nb = (len(prompt) + n + 15) // 16
    pool = torch.zeros(model.arch.num_layers, 2, nb, model.hkv, 16, 128, dtype=model.dtype, device=d)
    for _ in range(n):
        t = len(ids)
        pos = torch.arange(t, device=d)
        meta = AttnMetadata(True, pos.clone(), torch.arange(nb, dtype=torch.int32, device=d)[None],
                            torch.tensor([t], dtype=torch.int32, device=d),
                            torch.tensor([0, t], dtype=torch.int32, device=d), t)
        lg = model.compute_logits(model.forward(torch.tensor(ids, device=d), pos, meta, pool)[-1:])[0].float()
        top = torch.topk(lg, 2)
        toks.append(int(top.indices[0]))
        margins.append(float(top.values[0] - top.values[1]))
        ids.append(toks[-1])
    return toks, margins


def _tp_engine(rank: int, world: int, dev, steps: int = 16) -> Dict[str, Any]:
    """A tensor-parallel engine over every rank of the job (llama-mini, Megatron-split, hipGraph decode windows,
    the one-shot exchange in the row-parallel GEMM epilogue over the links): rank 0 serves three prompts, its
    greedy tokens are checked against a TP=1 no-cache recompute of the same full-size weights on rank 0's GPU
    (agreement up to the reference's first near-tie, as tests/test_engine_gpu.py does on one GPU)."""
    from src.config import EngineConfig
    from src.models.llama import CausalLM
    from src.models.presets import get_preset
    from src.parallel.tp import TPContext
    from src.parallel.tp_runner import build_tp_engine
    from src.preproc import SamplingParams

    cpu = dist.new_group(list(range(world)), backend="gloo") if dist.get_backend() != "gloo" else None
    tp = TPContext(rank=rank, world_size=world, cpu_group=cpu)
    cfg = EngineConfig(max_num_seqs=4, max_num_batched_tokens=256, num_kv_blocks=128, max_latency_ms=0.0,
                       use_cuda_graph=True, graph_batch_sizes=[1, 2, 4])
    obj = build_tp_engine("llama-mini", tp, str(dev), cfg=cfg, max_model_len=512, capture=True, full_init=True,
                          seed=3)
    res: Dict[str, Any] = {"preset": "llama-mini", "tp": world}
    if rank != 0:
        obj.follower_loop()
        return res
    obj.eos_token_id = None
    obj.generate(TP_PROMPTS[:1], SamplingParams(max_tokens=4))  # warm-up
    t0 = time.perf_counter()
    outs = obj.generate(TP_PROMPTS, SamplingParams(max_tokens=steps))
    res["generate_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    res["decode_steps"] = steps - 1
    res["graphs_replayed"] = bool(obj.runner.graphs)
    res["fused_exchange"] = bool(obj.model.decode_plan(4).get("tp_fused"))
    res["one_shot_error"] = bool(tp.car.error()) if tp.car is not None else None
    obj.runner.stop_followers()
    ref = CausalLM(get_preset("llama-mini"), str(dev), seed=3, max_position=512, full_init=True)
    agree = []
    for p, o in zip(TP_PROMPTS, outs):
        r, mg = _greedy_reference(ref, p, steps)
        ok = True
        for a, b, m in zip(o, r, mg):
            if m < 0.25:
                break
            if a != b:
                ok = False
                break
        agree.append(ok)
    res["tokens_agree_with_tp1"] = agree
    return res


def xgpu_probe(rank: int, world: int, dev, rccl: bool = True, group=None) -> Dict[str, Any]:
    """Run the three parts (each catching its own failure); returns rank 0's view (the same dict on every
    rank for the RCCL part; the KV hop reports every pair through ``per_rank``)."""
    out: Dict[str, Any] = {"world": world}
    t0 = time.perf_counter()
    if rccl:
        try:
            out["rccl_allreduce"] = _rccl_allreduce(dev, world, group)
        except Exception as e:  # noqa: BLE001 — reported, not raised: the bench result stands on its own
            out["rccl_allreduce"] = {"error": str(e)[:200]}
    try:
        out["ipc_allreduce"] = _ipc_allreduce(rank, world, dev, group, None if rccl else False)
    except Exception as e:  # noqa: BLE001
        out["ipc_allreduce"] = {"error": str(e)[:200]}
    try:
        out["kv_hop"] = _kv_hop(rank, world, dev, group)
    except Exception as e:  # noqa: BLE001
        out["kv_hop"] = {"error": str(e)[:200]}
    if 2 <= world <= 8:
        try:
            out["tp_engine"] = _tp_engine(rank, world, dev)
        except Exception as e:  # noqa: BLE001
            out["tp_engine"] = {"error": str(e)[:200]}
    out["probe_s"] = round(time.perf_counter() - t0, 2)
    return out


def main() -> None:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (a one-GPU rehearsal; gloo coordinates, no RCCL part)")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", 0 if a.same_device else local)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo" if a.same_device else "nccl")
    res = xgpu_probe(rank, world, dev, rccl=not a.same_device)
    if rank == 0:
        print(json.dumps({"bench": "xgpu_probe", **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
