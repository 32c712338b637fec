"""
Tensor-parallel execution of the engine: one process per GPU, rank 0 drives.

Rank 0 owns the scheduler, the KV block manager and the RPC front; every rank
owns its weight shard and its KV-head shard of the paged pool (the block ids
are the same on every rank, so one block table serves the whole group).

Step protocol (two messages per step):

1. an 8-word header ``[kind, a, b, c, d, payload words, 0, 0]`` broadcast on the
   host (gloo) group — followers read it without any GPU round trip;
2. ONE int64 payload with every input of the step packed back to back (token
   ids, positions, slots, context lengths, block-table rows, cu_q, last-token
   indices), built in pinned memory on rank 0, copied up once and broadcast over
   RCCL (xGMI); every rank unpacks it on the device into the runner's static
   input buffers.

Decode windows (round 6): a k-step window is ONE such message (kind WINDOW: the
first step's inputs, the window's [step counter, real rows] words and — when
the leader's device copies changed since its last decode message — the
sampling parameters); a continuation window
queued behind the running one is another (kind CONTINUE: the grown block
tables and first-step slots, plus its token-row base). Every rank replays its
graph k times; the graph's tail samples from the all-gathered logits
(bit-identical on every rank) and advances the inputs on the device, so the
followers stay in step without a message per step and the leader reads the
k x n tokens back once per window — the same host cost as the TP=1 engine's
queued windows (reference hot loop: /root/reference/src/worker.py:152).

Then all ranks run the identical forward — including replaying the same
captured decode hipGraph — and meet in the two per-layer all-reduces (one-shot
IPC kernel at decode sizes, fused with the residual add) and the logits
all-gather (one-shot IPC all-gather). Followers never synchronise with their
GPU: they can queue the next step as soon as its header arrives. Only rank 0
copies sampled token ids back to the host.

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

import numpy as np
import torch
import torch.distributed as dist

from src.config import EngineConfig
from src.engine.model_runner import KVPool, ModelRunner
from src.models.llama import CausalLM

logger = logging.getLogger(__name__)


class TPGroupFault(RuntimeError):
    """A collective of the TP group gave up waiting for a peer (dead or out of step): the step's
    outputs are poisoned and the group must be taken out of service as a unit."""


class TPModelRunner(ModelRunner):
    HEARTBEAT_S = 20.0
    # decode windows: the leader sends one message per k-step window (and per queued continuation), every rank
    # replays its captured graph k times and advances its own inputs on the device from the all-gathered
    # logits' samples (identical on every rank), so a window costs one host round trip on the leader only
    mirrors_windows = True
    HDR = 8

    def __init__(self, model: CausalLM, pool: KVPool, cfg: EngineConfig, max_model_len: int):
        super().__init__(model, pool, cfg, max_model_len)
        self.tp = model.tp
        self._last_sync = time.monotonic()
        self.h_hdr = torch.zeros(self.HDR, dtype=torch.int64)  # host (gloo) header
        cap = 3 * self.max_tokens + self.max_seqs * (self.bt_width + 3) + 1
        cap += 5 * self.max_seqs + 2  # a window's sampling parameters and step-counter words
        self.h_pkts = [torch.zeros(cap, dtype=torch.int64, pin_memory=self.is_cuda) for _ in range(2)]
        self._pkt_par = 0
        self.d_pkt = torch.zeros(cap, dtype=torch.int64, device=self.device)
        self.steps_synced = 0
        self.windows_synced = 0  # decode windows (and continuations) mirrored as one message each
        car = getattr(model.tp, "car", None)
        if car is not None and car.ranks_per_gpu > 4:
            # more than 4 ranks sharing ONE GPU (tests): queued windows keep every process's queues busy at once,
            # so the GPU time-slices them and each exchange waits for a peer's queue to be scheduled (one extra
            # context made the 8-rank group 5-10x slower; under the test runner it stalled): single steps there.
            # A node runs one rank per GPU.
            self.supports_multistep = False
        # the one-shot collectives' sticky error word (custom_allreduce ctl[2]), read back with the tokens
        self.h_fault = torch.zeros(1, dtype=torch.int32, pin_memory=self.is_cuda)

    # ------------------------------------------------------------ failure as a unit
    def _queue_fault_readback(self) -> None:
        super()._queue_fault_readback()
        car = self.tp.car
        if car is not None:
            self.h_fault.copy_(car.error_word(), non_blocking=True)

    def _raise_on_fault(self) -> None:
        super()._raise_on_fault()
        if self.tp.car is not None and int(self.h_fault[0]):
            raise TPGroupFault(f"TP rank {self.tp.rank}: a one-shot collective timed out waiting for a peer; "
                               "its outputs were poisoned and no token of this step is returned")

    # ------------------------------------------------------------ protocol
    KIND_WINDOW, KIND_CONTINUE = 4, 5

    def _fields(self, kind: int, a: int, b: int, d: int):
        """(device buffer, host staging buffer, rows) of the step's inputs, in payload order."""
        if kind == self.KIND_PREFILL:
            t, n, nd = a, b, d
            out = [(self.d_ids, self.h_ids, t), (self.d_pos, self.h_pos, t), (self.d_slots, self.h_slots, t),
                   (self.d_ctx, self.h_ctx, n), (self.d_bt, self.h_bt, n), (self.d_cu, self.h_cu, n + 1)]
            return out + [(self.d_last, self.h_last, nd)] if nd else out
        if kind in (self.KIND_DECODE, self.KIND_WINDOW):
            pad = b
            out = [(self.d_ids, self.h_ids, pad), (self.d_pos, self.h_pos, pad), (self.d_slots, self.h_slots, pad),
                   (self.d_ctx, self.h_ctx, pad), (self.d_bt, self.h_bt, pad)]
            if self.supports_multistep:  # the graph's input advance reads [step counter, real rows]
                out.append((self.d_ctl, self.h_ctl, 2))
            if d:
                # decode steps advance and SAMPLE on every rank: the followers' sampling parameters must equal the
                # leader's whenever its device copies changed (d = rows; prefill steps rewrite them too)
                out += [(self.d_temp, self.h_temp, d), (self.d_topk, self.h_topk, d), (self.d_topp, self.h_topp, d),
                        (self.d_seed, self.h_seed, d), (self.d_step, self.h_step, d)]
            return out
        if kind == self.KIND_CONTINUE:
            pad, par = a, d
            return [(self.d_bt, self.h_cbt[par], pad), (self.d_slots, self.h_cslots[par], pad)]
        return []

    def _pack(self, kind: int, a: int, b: int, d: int) -> int:
        # two pinned staging packets used in turn: the leader rewrites one only after the window whose H2D copy
        # read it has been waited for (at most a running window and its queued continuation are in flight)
        self._pkt_par ^= 1
        pkt = self.h_pkts[self._pkt_par].numpy()
        o = 0
        for _, hbuf, rows in self._fields(kind, a, b, d):
            src = hbuf[:rows].numpy().reshape(-1)
            if src.dtype == np.float32:
                src = src.view(np.int32)  # float parameters travel as their bit patterns
            pkt[o:o + src.size] = src
            o += src.size
        return o

    def _unpack(self, kind: int, a: int, b: int, d: int) -> None:
        o = 0
        for dbuf, _, rows in self._fields(kind, a, b, d):
            view = dbuf[:rows]
            n = view.numel()
            src = self.d_pkt[o:o + n]
            if view.dtype == torch.float32:
                view.copy_(src.to(torch.int32).view(torch.float32).view(view.shape))
            else:
                view.copy_(src.view(view.shape))  # int64 -> int32 where the buffer is int32
            o += n

    def _bcast(self, t: torch.Tensor) -> None:
        self.tp.broadcast(t, src=0)

    def _sync_step(self, kind: int, a: int = 0, b: int = 0, c: int = 0, d: int = 0) -> None:
        """Leader: header on the host group, then the packed payload (the leader's own device buffers
        were already filled by the runner's H2D copies, so it does not unpack)."""
        if not self.tp.enabled:
            return
        self._last_sync = time.monotonic()
        if kind in (self.KIND_DECODE, self.KIND_WINDOW) and self.supports_multistep:
            # mirror the sampling parameters whenever the leader rewrote its device copies since the last decode
            # message (a greedy window right after a prefill or a single step of another mix must not leave the
            # followers sampling with stale ones); d = the step's padded rows
            d = b if self._samp_dirty else 0
            self._samp_dirty = False
        nw = self._pack(kind, a, b, d)
        self.h_hdr.copy_(torch.tensor([kind, a, b, c, d, nw, 0, 0], dtype=torch.int64))
        self.tp.broadcast_host(self.h_hdr)
        if nw:
            self.d_pkt[:nw].copy_(self.h_pkts[self._pkt_par][:nw], non_blocking=self.is_cuda)
            self._bcast(self.d_pkt[:nw])
        self.steps_synced += 1

    def _sync_window(self, n: int, pad: int, k: int) -> None:
        """One message per k-step window: the first step's inputs (and the sampling parameters when the leader's
        changed); every rank then replays its graph k times and advances its inputs on the device."""
        self._sync_step(self.KIND_WINDOW, n, pad, k, 0)
        self.windows_synced += 1

    def _sync_continuation(self, par: int, pad: int, k: int, base: int) -> None:
        """A continuation window queued behind the running one: the grown block tables and first-step slots."""
        self._sync_step(self.KIND_CONTINUE, pad, k, base, par)
        self.windows_synced += 1

    def idle_tick(self) -> None:
        if self.tp.enabled and self.tp.rank == 0 and time.monotonic() - self._last_sync > self.HEARTBEAT_S:
            self._sync_step(self.KIND_HEARTBEAT)

    def stop_followers(self) -> None:
        if self.tp.enabled and self.tp.rank == 0:
            self._sync_step(self.KIND_STOP)

    @torch.inference_mode()
    def follower_loop(self) -> None:
        """Ranks > 0: mirror rank 0's steps until it sends STOP. No host-device synchronisation: the
        header arrives on the host group, the payload and the step's kernels are queued on the stream."""
        assert self.tp.rank != 0
        while True:
            self.tp.broadcast_host(self.h_hdr)
            kind, a, b, c, d, nw = (int(x) for x in self.h_hdr.tolist()[:6])
            if kind == self.KIND_STOP:
                return
            if kind == self.KIND_HEARTBEAT:
                continue
            if nw:
                self._bcast(self.d_pkt[:nw])
                self._unpack(kind, a, b, d)
            if kind == self.KIND_PREFILL:
                self._exec_prefill(a, b, c, d, True)
            elif kind == self.KIND_WINDOW:
                pad, k = b, c
                self._pre_embed(pad)
                g = self.graphs[pad]
                for _ in range(k):
                    g.replay()
                self.windows_synced += 1
            elif kind == self.KIND_CONTINUE:
                pad, k, base = a, b, c
                self.d_ctl[0:1].fill_(base)
                g = self.graphs[pad]
                for _ in range(k):
                    g.replay()
                self.windows_synced += 1
            else:
                self._exec_decode(a, b)
            self.steps_synced += 1


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
    # decode's row-parallel exchange: fused into the GEMM or its own launch, whichever this node's links run faster
    # (measured here, before the decode plan sizes the scratch and the graphs are captured)
    model.tp_exchange_calibration = model.calibrate_tp_exchange()
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
