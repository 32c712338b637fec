"""
Tensor-parallel execution of the engine: one process per GPU, rank 0 drives.

Rank 0 owns the scheduler, the KV block manager and the RPC front; every rank
owns its weight shard and its KV-head shard of the paged pool (the block ids
are the same on every rank, so one block table serves the whole group). Each
step rank 0 builds the inputs, copies them to its device and broadcasts a
6-int header plus the input tensors over RCCL (xGMI); then all ranks run the
identical forward — including replaying the same captured decode hipGraph —
and meet in the two per-layer all-reduces and the logits all-gather. Only
rank 0 copies sampled token ids back to the host.

Failure as a unit: the process group carries a finite collective timeout
(``init_tp(timeout_s=...)``) so a dead rank turns every peer's next collective
into an error (the leader's engine loop dies → its worker reports unhealthy →
the coordinator routes elsewhere) instead of a hang. An idle leader therefore
broadcasts a heartbeat step every ``HEARTBEAT_S`` so that followers parked in
their header broadcast never hit that timeout.
"""

from __future__ import annotations

import logging
import time
from typing import Optional

import torch
import torch.distributed as dist

from src.config import EngineConfig
from src.engine.model_runner import KVPool, ModelRunner
from src.models.llama import CausalLM

logger = logging.getLogger(__name__)


class TPModelRunner(ModelRunner):
    HEARTBEAT_S = 20.0

    def __init__(self, model: CausalLM, pool: KVPool, cfg: EngineConfig, max_model_len: int):
        super().__init__(model, pool, cfg, max_model_len)
        self.tp = model.tp
        self._last_sync = time.monotonic()
        self.hdr = torch.zeros(6, dtype=torch.int64, device=self.device)
        self.h_hdr = torch.zeros(6, dtype=torch.int64, pin_memory=self.is_cuda)

    def _bcast(self, t: torch.Tensor) -> None:
        self.tp.broadcast(t, src=0)

    def _sync_step(self, kind: int, a: int = 0, b: int = 0, c: int = 0, d: int = 0) -> None:
        if not self.tp.enabled:
            return
        self._last_sync = time.monotonic()
        self.h_hdr.copy_(torch.tensor([kind, a, b, c, d, 0], dtype=torch.int64))
        self.hdr.copy_(self.h_hdr, non_blocking=self.is_cuda)
        self._bcast(self.hdr)
        self._bcast_inputs(kind, a, b, c, d)

    def _bcast_inputs(self, kind: int, a: int, b: int, c: int, d: int) -> None:
        if kind == self.KIND_PREFILL:
            t, n, nd = a, b, d
            for buf in (self.d_ids[:t], self.d_pos[:t], self.d_slots[:t], self.d_ctx[:n], self.d_bt[:n],
                        self.d_cu[: n + 1]):
                self._bcast(buf)
            if nd:
                self._bcast(self.d_last[:nd])
        elif kind == self.KIND_DECODE:
            pad = b
            for buf in (self.d_ids[:pad], self.d_pos[:pad], self.d_slots[:pad], self.d_ctx[:pad],
                        self.d_bt[:pad]):
                self._bcast(buf)

    def idle_tick(self) -> None:
        if self.tp.enabled and self.tp.rank == 0 and time.monotonic() - self._last_sync > self.HEARTBEAT_S:
            self._sync_step(self.KIND_HEARTBEAT)

    def stop_followers(self) -> None:
        if self.tp.enabled and self.tp.rank == 0:
            self._sync_step(self.KIND_STOP)

    @torch.inference_mode()
    def follower_loop(self) -> None:
        """Ranks > 0: mirror rank 0's steps until it sends STOP."""
        assert self.tp.rank != 0
        while True:
            self._bcast(self.hdr)
            kind, a, b, c, d, _ = (int(x) for x in self.hdr.tolist())
            if kind == self.KIND_STOP:
                return
            if kind == self.KIND_HEARTBEAT:
                continue
            self._bcast_inputs(kind, a, b, c, d)
            if kind == self.KIND_PREFILL:
                self._exec_prefill(a, b, c, d, True)
            else:
                self._exec_decode(a, b)
            if self.is_cuda:
                torch.cuda.current_stream(self.device).synchronize()


def agree_num_blocks(n: int, tp) -> int:
    """Every rank must use the same block ids: take the minimum."""
    if not tp.enabled or getattr(tp, "probe", False):
        return n
    dev = "cuda" if torch.cuda.is_available() and dist.get_backend(tp.group) == "nccl" else "cpu"
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=tp.group)
    return int(t.item())


def build_tp_engine(preset: str, tp, device, cfg: Optional[EngineConfig] = None, max_model_len: int = 4096,
                    seed: int = 0, capture: bool = True, dtype=torch.bfloat16, full_init: bool = False,
                    moe_parallel: str = "tp", sequence_parallel: bool = False, **arch_overrides):
    """Construct the per-rank pieces. Rank 0 gets an :class:`LLMEngine`
    (scheduler + RPC-facing API) whose runner broadcasts steps; other ranks get
    a :class:`TPModelRunner` on which to call :meth:`follower_loop`."""
    from src.engine.llm_engine import LLMEngine, plan_kv_blocks
    from src.models.loader import arch_from_hf_config, is_hf_checkpoint, load_checkpoint
    from src.models.presets import get_preset

    ckpt = is_hf_checkpoint(preset)  # `preset` may be a local HF checkpoint directory
    arch = arch_from_hf_config(preset, **arch_overrides) if ckpt else get_preset(preset, **arch_overrides)
    cfg = cfg or EngineConfig()
    if torch.device(device).type == "cuda":
        tp.enable_custom_allreduce()  # decode-sized all-reduces: one xGMI hop instead of RCCL's ring
    model = CausalLM(arch, device, dtype=dtype, tp=tp, seed=seed, max_position=max(max_model_len, 16),
                     full_init=full_init, moe_parallel=moe_parallel, sequence_parallel=sequence_parallel)
    if ckpt:
        load_checkpoint(model, preset)  # every rank streams the shards and keeps its own slice
    nblocks = agree_num_blocks(plan_kv_blocks(arch, model, cfg, model.device), tp)
    cfg = EngineConfig(**{**cfg.__dict__, "num_kv_blocks": nblocks})
    if tp.rank == 0:
        eng = LLMEngine(model, cfg, max_model_len, runner_cls=TPModelRunner)
        if capture:
            eng.runner.capture_graphs()
        return eng
    pool = KVPool(arch.num_layers, nblocks, model.hkv, cfg.block_size, arch.head_dim, model.device, dtype=dtype)
    runner = TPModelRunner(model, pool, cfg, min(max_model_len, model.max_position))
    if capture:
        runner.capture_graphs()
    return runner
