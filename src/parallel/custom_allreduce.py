"""
One-shot all-reduce over xGMI for tensor-parallel decode (``csrc/kernels/allreduce.hip``).

RCCL's ring/tree all-reduce is the right tool for large prefill messages, but a decode step of
Llama-3-70B at TP=8 issues 160 all-reduces of only 512 KiB (``[32, 8192]`` bf16); there the
latency of W-1 protocol hops dominates. Every MI355X of a node has a direct xGMI link to each of
the others, so this path does ONE hop: each rank publishes its input in an IPC-shared staging
buffer and every rank reads all W inputs over the 7 links at once and sums them in rank order
(bit-identical on every rank). Messages above ``max_bytes`` and every non-bf16 tensor fall back to
RCCL.

Setup is collective over the TP group (any backend: the IPC handles travel as Python objects):
each rank allocates an uncached staging buffer ``[2][cap]`` and an uncached flag page, exchanges
IPC handles and opens its peers'. The launch is hipGraph-capturable (its epoch is a device word).

The same code validates on ONE GPU with several processes sharing it (the peers' "remote" memory
is then local); ``tests/test_custom_allreduce_gpu.py`` does that.
"""

from __future__ import annotations

import logging
from typing import List, Optional

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)

MAX_RANKS = 8
MAX_BLOCKS = 64                 # rows of the fused all-reduce + residual kernel (one workgroup per row)
SIG_BLOCKS = 256                # flag slots per parity and rank (csrc CAR_MAX_BLOCKS): workgroups / GEMM tiles
SIG_BYTES = 2 * SIG_BLOCKS * MAX_RANKS * 4


def _kern():
    from src import _C

    return _C


def residency_margin(cus: int) -> int:
    """Workgroup slots rule (a) of :func:`fused_exchange_ok` keeps free: 1/16 of the CUs (16 on MI355X)."""
    return max(4, cus // 16)


def fused_exchange_ok(n_tiles: int, grid: int, per_cu: int, ranks_per_gpu: int, cus: int) -> bool:
    """Residency rule of the exchange fused into the row-parallel decode GEMM. Only a column tile's last-arriving
    workgroup waits for the peers (one flag slot per tile), so a launch holds at most ``n_tiles`` waiting
    workgroups per rank. The grid always drains when either

    (a) every workgroup of every rank sharing the GPU is resident at once WITH a margin: ``grid`` x ranks <=
        ``per_cu`` x CUs - margin, where ``per_cu`` is the kernel's occupancy (hipOccupancyMaxActiveBlocksPerMultiprocessor
        on the exact instantiation: LDS ring, registers) — so a few CUs held by another stream's kernel, or a CU
        mask, still leave room for the whole grid; or
    (b) the waiting workgroups can hold at most HALF the CUs, so the others always find a CU and finish.

    When neither holds the caller keeps the separate all-reduce launch (never a spin that could only end at the
    bounded wait). The 70B TP=8 shard's o / down at 32 rows (wr = 32: 256 tiles, grid 256, one workgroup per CU
    with the full LDS ring) fail both and take the half-LDS ring (two per CU: 256 <= 512 - 16)."""
    if not 0 < n_tiles <= SIG_BLOCKS:
        return False
    if ranks_per_gpu > 1:
        # ranks sharing ONE GPU (the one-GPU tests, never a node): the GPU time-slices the processes' queues and
        # another rank's next kernel (a full-LDS GEMM ring) needs a whole CU, so small-ring waiters spread one per CU
        # would leave none (measured: 8 ranks with half-ring waiters stalled until the bounded spin). These groups
        # keep the round-5 rule that the one-GPU suite has validated: one workgroup per CU, no margin.
        return (0 < grid and grid * ranks_per_gpu <= cus) or n_tiles * ranks_per_gpu * 2 <= cus
    if grid > 0 and per_cu > 0 and grid * ranks_per_gpu <= per_cu * cus - residency_margin(cus):
        return True
    return n_tiles * ranks_per_gpu * 2 <= cus


class CustomAllReduce:
    """IPC-mapped one-shot all-reduce for one TP group (2..8 ranks on one node)."""

    def __init__(self, rank: int, world: int, group=None, max_bytes: int = 8 << 20, blocks: int = 48):
        if not 2 <= world <= MAX_RANKS:
            raise ValueError("custom all-reduce needs 2..8 ranks")
        self.rank, self.world, self.group = rank, world, group
        self.max_bytes = max_bytes
        self.cap = max_bytes // 2            # bf16 elements per half of the double buffer
        self.blocks = min(blocks, MAX_BLOCKS)
        k = _kern()
        self._own = [k.car_alloc(2 * max_bytes), k.car_alloc(SIG_BYTES)]
        # [epoch, ticket, error] words: ordinary device memory (device-scope atomics), zeroed once
        self._ctl = torch.zeros(4, dtype=torch.int32, device=torch.device("cuda", torch.cuda.current_device()))
        self.ctl = self._ctl.data_ptr()
        handles = [k.car_handle(self._own[0]), k.car_handle(self._own[1])]
        allh: List[Optional[list]] = [None] * world
        dist.all_gather_object(allh, handles, group=group)
        self._opened: List[int] = []
        self.bufs: List[int] = []
        self.sigs: List[int] = []
        for p in range(world):
            if p == rank:
                self.bufs.append(self._own[0])
                self.sigs.append(self._own[1])
            else:
                b, s = k.car_open(allh[p][0]), k.car_open(allh[p][1])
                self._opened += [b, s]
                self.bufs.append(b)
                self.sigs.append(s)
        # how many ranks of the group share one GPU (tests run 2..8 ranks on one GPU; a node runs one per GPU):
        # bounds the waiting workgroups of the fused row-parallel GEMM (fused_ok)
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        key = str(getattr(props, "uuid", "") or "") or \
            f"{getattr(props, 'pci_domain_id', '?')}:{getattr(props, 'pci_bus_id', '?')}:{getattr(props, 'pci_device_id', '?')}"
        keys: List[Optional[str]] = [None] * world
        dist.all_gather_object(keys, key, group=group)
        self.ranks_per_gpu = max(keys.count(k) for k in keys)
        self.cus = int(props.multi_processor_count)
        dist.barrier(group=group)  # every rank's pages are open before anyone signals into them

    def can_run(self, t: torch.Tensor) -> bool:
        n = t.numel()
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and n % 8 == 0
                and 0 < n * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sum ``t`` over the group (in place unless ``out`` is given) on the current stream."""
        out = t if out is None else out
        _kern().car_all_reduce(t, out, self.rank, self.bufs, self.sigs, self.ctl, self.cap, self.blocks)
        return out

    def can_run_gather(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.is_contiguous()
                and t.shape[1] % 8 == 0 and 0 < t.numel() * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        """[rows, cols] per rank -> [rows, world * cols] (rank-major along the last dim), one launch."""
        out = torch.empty(t.shape[0], self.world * t.shape[1], dtype=t.dtype, device=t.device)
        _kern().car_all_gather(t, out, self.rank, self.bufs, self.sigs, self.ctl, self.cap, self.blocks)
        return out

    def can_run_residual(self, x: torch.Tensor, resid: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.shape[0] <= MAX_BLOCKS
                and x.shape[1] % 8 == 0 and 2 * x.numel() <= self.max_bytes and x.is_contiguous()
                and resid.is_contiguous() and resid.shape == x.shape and x.data_ptr() % 16 == 0
                and resid.data_ptr() % 16 == 0)

    def all_reduce_residual(self, x: torch.Tensor, resid: torch.Tensor, ssp: torch.Tensor) -> None:
        """resid += sum over the group of x (bf16, in place), ssp[row] = that row's sum of squares of the
        new residual — all-reduce and residual_add_sumsq in one launch (decode rows, <= 64)."""
        _kern().car_all_reduce_residual(x, resid, ssp, self.rank, self.bufs, self.sigs, self.ctl, self.cap)

    def fused_ok(self, n_tiles: int, grid: int = 0, per_cu: int = 0) -> bool:
        """Whether the row-parallel decode GEMM may carry the exchange in its epilogue (gemm_decode_car); see
        :func:`fused_exchange_ok` (``per_cu``: the launch's resident workgroups per CU, ops.gd_occupancy).
        ``DIE_TP_FUSED=0`` keeps the separate all-reduce launch. The answer depends only on the group's layout and
        the shape, so every rank agrees."""
        import os

        if os.environ.get("DIE_TP_FUSED", "1") == "0":
            return False
        return fused_exchange_ok(n_tiles, grid, per_cu, self.ranks_per_gpu, self.cus)

    def row_parallel_residual(self, x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor, ssp: torch.Tensor,
                              counters: torch.Tensor, wr: int, kc: int, sk: int, tiled: bool,
                              half_ring: bool = False) -> None:
        """resid += sum over the group of x @ w^T (this rank's K shard), ssp [N / wr, 128] = per-tile row sums of
        squares of the new residual: ONE launch (decode GEMM mode 3 whose tiles' last arrivers run the one-shot
        exchange). Every rank must make the same call."""
        from src import ops

        m, n = x.shape[0], w.shape[0]
        slab = torch.empty(sk, m, n, dtype=torch.float32, device=x.device)
        _kern().gemm_decode_car(slab, x, w, 3 | (32 if tiled else 0) | (64 if half_ring else 0), wr, kc, sk,
                                ops.DECODE_GEMM_NT, resid, ssp,
                                counters, self.rank, self.bufs, self.sigs, self.ctl, self.cap)

    def read_ctl(self) -> List[int]:
        """[epoch, ticket, error] control words (synchronising host read)."""
        return list(_kern().car_read_words(self.ctl, 3))

    def error(self) -> bool:
        """True once a call gave up waiting for a peer (a dead rank, or a rank out of step). The sticky
        word stays set: that call's output was poisoned (NaN) and every later call fails fast."""
        return bool(self.read_ctl()[2])

    def error_word(self) -> torch.Tensor:
        """The sticky error word as a 1-element device tensor (for a non-blocking readback)."""
        return self._ctl[2:3]

    def close(self) -> None:
        k = _kern()
        for p in self._opened:
            try:
                k.car_close(p)
            except Exception:  # pragma: no cover - teardown
                pass
        for p in self._own:
            try:
                k.car_release(p)
            except Exception:  # pragma: no cover
                pass
        self._opened, self._own = [], []

