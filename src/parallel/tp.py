"""
Tensor parallelism over RCCL (torch.distributed ``"nccl"`` backend = RCCL on
ROCm), one process per GPU.

Megatron-style split, chosen for xGMI's point-to-point links: per decoder layer
exactly two all-reduces (after the row-parallel ``o_proj`` and ``down_proj``),
each of ``tokens x hidden`` bf16 — for 70B TP=8 decode at batch 32 that is
512 KiB, small enough that RCCL picks its low-latency one-shot/LL protocols
over the 7 xGMI links. QKV and gate/up are column-parallel (each rank owns
whole heads / a contiguous slice of the FFN), the LM head is vocab-parallel
with one all-gather of the logits, the embedding is replicated (2 GiB for
70B — trivial against 288 GB of HBM, and it saves a collective per step).
Decode-sized all-reduces (<= 8 MiB bf16) take the one-shot IPC kernel of
``custom_allreduce.py`` (one xGMI hop on all 7 links at once, bit-identical
on every rank); prefill-sized ones stay on RCCL.
On CPU the same code runs on ``gloo`` for tests.
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class TPContext:
    rank: int = 0
    world_size: int = 1
    group: Optional[object] = None
    car: Optional[object] = None  # CustomAllReduce (one-shot IPC all-reduce) once enabled
    # host-side group for the step protocol's headers (gloo): followers learn each step's kind and
    # sizes without a GPU round trip (None = the default group, when that is gloo already)
    cpu_group: Optional[object] = None
    # test hook: run the collectives even at world_size 1 (a one-rank RCCL group pins the RCCL branches'
    # shapes and dtypes on a one-GPU box; tests/test_rccl_gpu.py)
    force_collectives: bool = False
    # the group's measured choice between the exchange fused into the row-parallel GEMM and the separate one-shot
    # launch (CausalLM.calibrate_tp_exchange at engine build; None: not measured, the fused form where it may run)
    fused_preferred: Optional[bool] = None

    def src_rank(self) -> int:
        """Global rank of this group's rank 0 (the ``src`` of broadcasts)."""
        if self.group is None:
            return 0
        return dist.get_global_rank(self.group, 0)

    def enable_custom_allreduce(self, max_bytes: int = 8 << 20) -> bool:
        """Collective over the group: set up the one-shot IPC all-reduce (src/parallel/custom_allreduce.py)
        for GPU tensors of up to ``max_bytes`` — the decode-sized messages; larger ones stay on RCCL.
        ``DIE_CUSTOM_AR=0`` keeps everything on RCCL. Every rank must make the same call."""
        if not self.enabled or self.car is not None:
            return self.car is not None
        if os.environ.get("DIE_CUSTOM_AR", "1") == "0" or not torch.cuda.is_available() or self.world_size > 8:
            return False
        from src.parallel.custom_allreduce import CustomAllReduce

        self.car = CustomAllReduce(self.rank, self.world_size, self.group, max_bytes=max_bytes)
        return True

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.force_collectives

    def shard(self, n: int) -> int:
        if n % self.world_size:
            raise ValueError(f"{n} not divisible by tp={self.world_size}")
        return n // self.world_size

    def kv_heads(self, n_kv: int) -> int:
        """KV heads per rank: split when divisible, replicate when tp > n_kv."""
        if n_kv >= self.world_size:
            return self.shard(n_kv)
        if self.world_size % n_kv:
            raise ValueError("tp must be a multiple of num_kv_heads when tp > num_kv_heads")
        return 1

    def _staged(self, t: torch.Tensor) -> bool:
        """GPU tensors over a gloo group (e.g. several ranks validating TP on one GPU): stage the
        collective through host memory in fp32. The RCCL path never takes this branch."""
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.enabled:
            car = self.car
            # the choice depends only on dtype and size, so every rank takes the same path
            if car is not None and t.is_cuda and t.dtype == torch.bfloat16 and t.numel() % 8 == 0 \
                    and 0 < 2 * t.numel() <= car.max_bytes:
                if t.is_contiguous() and t.data_ptr() % 16 == 0:
                    car.all_reduce(t)
                else:
                    t.copy_(car.all_reduce(t.contiguous().clone()))
            elif self._staged(t):
                c = t.float().cpu()
                dist.all_reduce(c, group=self.group)
                t.copy_(c)
            else:
                dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_residual(self, x: torch.Tensor, resid: torch.Tensor, ssp: torch.Tensor) -> None:
        """resid += all_reduce(x); ssp[0, row] = sum of squares of the new residual row (the next norm's
        statistics). One fused launch on the one-shot IPC path, else all-reduce + residual_add_sumsq.
        The choice depends only on shapes, so every rank takes the same path."""
        car = self.car
        if self.enabled and car is not None and car.can_run_residual(x, resid):
            car.all_reduce_residual(x, resid, ssp)
            return
        from src import ops

        ops.residual_add_sumsq(resid, self.all_reduce(x), ssp)

    def fused_row_parallel(self, n_tiles: int, grid: int = 0, per_cu: int = 0) -> bool:
        """Whether a row-parallel decode projection with ``n_tiles`` column tiles (``grid`` workgroups, ``per_cu``
        resident per CU) runs as ONE launch: the decode GEMM whose tiles' last arrivers exchange their partials
        one-shot and update the residual (:meth:`row_parallel_residual`), instead of GEMM + all-reduce/residual
        kernel. Needs the IPC path and the residency rule (custom_allreduce.fused_exchange_ok)."""
        return (self.enabled and self.car is not None and self.fused_preferred is not False
                and self.car.fused_ok(n_tiles, grid, per_cu))

    def row_parallel_residual(self, x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor, ssp: torch.Tensor,
                              counters: torch.Tensor, wr: int, kc: int, sk: int, tiled: bool = False,
                              half_ring: bool = False) -> None:
        """resid += all_reduce(x @ w^T) and the next norm's per-tile statistics, in one launch
        (see :meth:`fused_row_parallel`, which the caller checked with this tile's ``n_tiles``)."""
        self.car.row_parallel_residual(x, w, resid, ssp, counters, wr, kc, sk, tiled, half_ring)

    # --- sequence parallelism (Megatron-SP): the all-reduce split into its two halves around the
    # token-sharded norms. Rows = tokens, padded by the caller to a multiple of world_size.
    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        """[T, H] partial sums -> this rank's [T / W, H] rows of the total."""
        if not self.enabled:
            return t
        n = t.shape[0] // self.world_size
        if dist.get_backend(self.group) == "gloo":  # gloo has no reduce-scatter: all-reduce + slice
            full = self.all_reduce(t.clone())
            return full[self.rank * n:(self.rank + 1) * n].contiguous()
        out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
        return out

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """This rank's [T / W, H] rows -> [T, H] (rank-major)."""
        if not self.enabled:
            return t
        if dist.get_backend(self.group) == "gloo":
            c = t.float().cpu().contiguous() if t.is_cuda else t.contiguous()
            parts = [torch.empty_like(c) for _ in range(self.world_size)]
            dist.all_gather(parts, c, group=self.group)
            return torch.cat(parts, 0).to(t.device, t.dtype)
        out = torch.empty((t.shape[0] * self.world_size,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate the per-rank shards [rows, cols] along the last dim (the vocab-parallel logits):
        one launch of the one-shot IPC all-gather for decode-sized tensors (hipGraph-capturable on any
        backend), else ONE all_gather_into_tensor into [W, rows, cols] and a permute."""
        if not self.enabled:
            return t
        car = self.car
        if car is not None and t.dim() == 2 and car.can_run_gather(t):
            return car.all_gather_last(t)
        if self._staged(t) or dist.get_backend(self.group) == "gloo":  # gloo: list form (host-staged for GPU tensors)
            c = t.float().cpu().contiguous() if t.is_cuda else t.contiguous()
            parts = [torch.empty_like(c) for _ in range(self.world_size)]
            dist.all_gather(parts, c, group=self.group)
            return torch.cat(parts, dim=-1).to(t.device, t.dtype)
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out.movedim(0, -2).reshape(*t.shape[:-1], self.world_size * t.shape[-1])

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.enabled:
            src = self.src_rank() if src == 0 else src
            if self._staged(t):
                c = t.cpu()
                dist.broadcast(c, src=src, group=self.group)
                t.copy_(c)
            else:
                dist.broadcast(t, src=src, group=self.group)
        return t

    def broadcast_host(self, t: torch.Tensor) -> torch.Tensor:
        """Broadcast a small CPU tensor from rank 0 over the host group (no GPU involvement)."""
        if self.enabled:
            dist.broadcast(t, src=self.src_rank(), group=self.cpu_group)
        return t


class ShardProbeTP(TPContext):
    """Rank 0's shard of a TP=``world_size`` model in ONE process, collectives replaced by local
    stand-ins (all-reduce = identity, all-gather = ``world_size`` copies of the local shard,
    broadcast = nothing). Every GEMM, attention and norm runs at the real per-rank shapes, so the
    step time is the per-rank COMPUTE of the TP configuration (e.g. Llama-3-70B TP=8 on one GPU,
    bench/tp_probe.py); the collectives' cost is not in it, and the tokens are meaningless."""

    probe = True

    def __init__(self, world_size: int):
        super().__init__(rank=0, world_size=world_size, group=None)

    def enable_custom_allreduce(self, max_bytes: int = 8 << 20) -> bool:
        return False

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def all_reduce_residual(self, x: torch.Tensor, resid: torch.Tensor, ssp: torch.Tensor) -> None:
        from src import ops

        ops.residual_add_sumsq(resid, x, ssp)  # the non-fused path's local launch

    def fused_row_parallel(self, n_tiles: int, grid: int = 0, per_cu: int = 0) -> bool:
        # the fused epilogue's local form, under the same residency rule as a real group of one rank per GPU
        # (so the probe runs the tiles a node would run; DIE_TP_FUSED=0: the separate-launch form, for A/B)
        if os.environ.get("DIE_TP_FUSED", "1") == "0":
            return False
        from src.parallel.custom_allreduce import fused_exchange_ok

        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count \
            if torch.cuda.is_available() else 256
        return fused_exchange_ok(n_tiles, grid, per_cu, 1, cus)

    def row_parallel_residual(self, x, w, resid, ssp, counters, wr, kc, sk, tiled=False, half_ring=False) -> None:
        from src import ops

        # the one-launch row-parallel projection minus its exchange (mode 3 on the K shard); the exchange's
        # xGMI cost is not in the probe
        ops.linear_slab_residual(x, w, resid, ssp, counters, wr, sk, tiled=tiled, kc=kc, half_ring=half_ring)

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        n = t.shape[0] // self.world_size
        return t[:n].contiguous()

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        return torch.cat([t] * self.world_size, 0)

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        return torch.cat([t] * self.world_size, dim=-1)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t

    def broadcast_host(self, t: torch.Tensor) -> torch.Tensor:
        return t


_TP: Optional[TPContext] = None


def init_tp(tp_size: Optional[int] = None, backend: Optional[str] = None,
            timeout_s: Optional[float] = None) -> TPContext:
    """Initialise (or reuse) the default process group and return the TP
    context. Reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from the
    environment (torchrun). ``timeout_s`` bounds every collective (a dead rank
    then fails its peers instead of hanging them; serving leaders send
    heartbeats while idle, see tp_runner)."""
    global _TP
    world = int(os.environ.get("WORLD_SIZE", "1"))
    tp = tp_size or world
    if tp == 1:
        _TP = TPContext()
        return _TP
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        kw = {"timeout": datetime.timedelta(seconds=timeout_s)} if timeout_s else {}
        dist.init_process_group(backend=backend, **kw)
    rank = dist.get_rank()
    world_all = dist.get_world_size()
    starts = range(0, world_all, tp)
    if world_all == tp:
        group = None
    else:
        # consecutive ranks form a TP group (GPUs of one xGMI-connected node)
        groups = [dist.new_group(list(range(s, s + tp))) for s in starts]
        group = groups[rank // tp]
    cpu_group = group
    if dist.get_backend() != "gloo":  # step headers travel on a host (gloo) group: no GPU sync to read them
        cpu_groups = [dist.new_group(list(range(s, s + tp)), backend="gloo") for s in starts]
        cpu_group = cpu_groups[rank // tp]
    _TP = TPContext(rank=rank % tp, world_size=tp, group=group, cpu_group=cpu_group)
    return _TP


def get_tp() -> TPContext:
    return _TP or TPContext()
