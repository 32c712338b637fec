"""
LLMEngine: model + paged KV pool + scheduler + runner for one worker (one GPU,
or one TP group driven from its rank 0).

    engine = LLMEngine.from_preset("llama3-8b", device="cuda:0")
    engine.add_request("r1", prompt_ids, SamplingParams(max_tokens=128))
    while engine.has_work(): finished = engine.step()

HBM budget (288 GB per MI355X): weights are created first, then the KV pool
takes ``gpu_memory_fraction`` of what is left after an activation reserve
sized from ``max_num_batched_tokens`` — for Llama-3-8B that is ≈1.9 M tokens of
KV (128 KiB/token), so prefix blocks stay cached long after their requests
finish and LRU/TTL eviction only starts under real memory pressure.
"""

from __future__ import annotations

import collections
import dataclasses
import logging
import time
from typing import Callable, Dict, List, Optional

import torch

from src.config import EngineConfig
from src.engine.block_manager import KVBlockManager
from src.engine.model_runner import KVPool, ModelRunner
from src.engine.scheduler import Scheduler, SchedulerOutput
from src.engine.sequence import Sequence, SeqStatus
from src.models.llama import CausalLM
from src.models.presets import ArchConfig, get_preset
from src.parallel.tp import TPContext
from src.preproc import SamplingParams

logger = logging.getLogger(__name__)


def plan_kv_blocks(arch: ArchConfig, model: CausalLM, cfg: EngineConfig, device: torch.device) -> int:
    if cfg.num_kv_blocks:
        return cfg.num_kv_blocks
    per_block = KVPool.bytes_per_block(arch.num_layers, model.hkv, cfg.block_size, arch.head_dim)
    if device.type != "cuda":
        return 512
    free, total = torch.cuda.mem_get_info(device)
    h = arch.hidden_size
    inter = model.inter * (arch.top_k if arch.is_moe else 1)
    t = cfg.max_num_batched_tokens
    # activations of one prefill step (qkv, attn, gate_up, act, residual ...) + logits + slack
    act = t * (3 * h + (model.hq + 2 * model.hkv) * arch.head_dim + 3 * inter) * 2
    act += cfg.max_num_seqs * arch.vocab_size * 4 + (2 << 30)
    budget = min(free - act, cfg.gpu_memory_fraction * total - (total - free) - act)
    return max(16, int(budget // per_block))


def choose_decode_weight_layout(model, cfg: EngineConfig, device: torch.device, buckets) -> str:
    """"tiled" or "single" (EngineConfig.decode_weight_layout): "auto" keeps the tile-order copies unless the KV
    pool is the constraint — cfg.kv_capacity_priority, or an explicit num_kv_blocks that the HBM left after the
    copies cannot hold (/root/reference/src/kvstore.py:82-102: capacity is what the LRU evicts for)."""
    mode = getattr(cfg, "decode_weight_layout", "auto")
    if mode in ("tiled", "single"):
        return mode
    if mode != "auto":
        raise ValueError(f"decode_weight_layout must be auto / tiled / single, not {mode!r}")
    if getattr(cfg, "kv_capacity_priority", False):
        return "single"
    if cfg.num_kv_blocks and device.type == "cuda" and hasattr(model, "decode_copy_bytes"):
        extra = model.decode_copy_bytes(buckets)
        if extra:
            fits = plan_kv_blocks(model.arch, model, EngineConfig(**{**cfg.__dict__, "num_kv_blocks": None}), device)
            per_block = KVPool.bytes_per_block(model.arch.num_layers, model.hkv, cfg.block_size, model.arch.head_dim)
            if cfg.num_kv_blocks > fits - extra // per_block:
                return "single"
    return "tiled"


class LLMEngine:
    def __init__(self, model: CausalLM, cfg: EngineConfig, max_model_len: int, eos_token_id: Optional[int] = 2,
                 runner_cls=ModelRunner):
        self.model = model
        self.arch = model.arch
        self.cfg = cfg
        self.device = model.device
        self.max_model_len = min(max_model_len, model.max_position)
        self.eos_token_id = eos_token_id
        if self.device.type == "cuda" and getattr(cfg, "tuned_gemm_table", True):
            from src.ops.gemm_table import enable_prefill_gemm_table

            enable_prefill_gemm_table(self.device)
        self.decode_weight_layout = "row-major"
        if hasattr(model, "pack_decode_weights") and hasattr(model, "decode_buckets"):
            # the decode GEMMs' tile-order weight copies are made before the KV pool takes the free HBM — unless
            # the KV pool is the constraint (EngineConfig.decode_weight_layout)
            buckets = model.decode_buckets(cfg.max_num_seqs)
            if choose_decode_weight_layout(model, cfg, self.device, buckets) == "single":
                model.tiled_decode_weights = False
            if model.pack_decode_weights(buckets):
                self.decode_weight_layout = "tiled"
            logger.info("decode weights: %s (%s)", self.decode_weight_layout,
                        f"+{model.decode_copy_bytes(buckets) / 2**30:.1f} GiB of tile-order copies"
                        if self.decode_weight_layout == "tiled" else "one copy, HBM left to the KV pool")
        if hasattr(model, "pack_lm_head"):
            model.pack_lm_head()
        nblocks = plan_kv_blocks(self.arch, model, cfg, self.device)
        self.pool = KVPool(self.arch.num_layers, nblocks, model.hkv, cfg.block_size, self.arch.head_dim,
                           self.device, dtype=model.dtype)
        self.blocks = KVBlockManager(nblocks, cfg.block_size, cfg.enable_prefix_caching, cfg.kv_block_ttl_s)
        self.runner = runner_cls(model, self.pool, cfg, self.max_model_len)
        # host swap space for preempted sequences (single-process runners only: a TP group would
        # have to mirror every swap on its followers, so it always recomputes)
        per_block = KVPool.bytes_per_block(self.arch.num_layers, model.hkv, cfg.block_size, self.arch.head_dim)
        swap_blocks = 0
        if cfg.preemption_mode != "recompute" and getattr(self.runner, "supports_swap", False):
            swap_blocks = int(cfg.swap_space_gib * 2**30 // per_block)
        self.scheduler = Scheduler(cfg, self.blocks, self.max_model_len, swap_capacity_blocks=swap_blocks)
        self.seqs: Dict[str, Sequence] = {}
        self._step_est = 0.004  # EMA of one decode step (s): sizes windows that must end by a deadline
        self._pf_tok_est = 0.0  # EMA of prefill time per prompt token (s), 0 until the first prefill step
        self.load_snapshot: dict = {}
        # disaggregated decode: imported prompts join the running batch directly (no waiting queue), so a burst of
        # imports would otherwise join one decode WINDOW late each; while imports keep arriving (the last one less
        # than cfg.import_settle_ms ago) the engine runs single steps so the next import joins at the next step
        self._import_settle_s = float(cfg.import_settle_ms) / 1e3
        self._last_import = -1e9
        # open-loop arrivals: times of the requests that arrived while sequences were decoding (a closed-loop wave
        # arrives while the engine is idle and is not counted); see EngineConfig.arrival_window_ms
        self._dec_arrivals: "collections.deque[float]" = collections.deque(maxlen=64)
        self._arrival_lookback_s = float(cfg.arrival_window_ms) / 1e3
        self.stats = {"prompt_tokens": 0, "generated_tokens": 0, "finished": 0, "prefill_time": 0.0,
                      "decode_time": 0.0, "steps": 0, "prefix_hit_tokens": 0}
        logger.info("KV pool: %d blocks x %d tokens = %.1f GiB (%d tokens)", nblocks, cfg.block_size,
                    self.pool.nbytes / 2**30, nblocks * cfg.block_size)

    @classmethod
    def from_preset(cls, preset: str, device="cuda:0", cfg: Optional[EngineConfig] = None, max_model_len: int = 4096,
                    tp: Optional[TPContext] = None, seed: int = 0, capture: bool = True, dtype=torch.bfloat16,
                    **arch_overrides):
        arch = get_preset(preset, **arch_overrides)
        cfg = cfg or EngineConfig()
        model = CausalLM(arch, device, dtype=dtype, tp=tp, seed=seed, max_position=max(max_model_len, 16))
        eng = cls(model, cfg, max_model_len)
        if capture:
            eng.runner.capture_graphs()
        return eng

    @classmethod
    def from_pretrained(cls, path: str, device="cuda:0", cfg: Optional[EngineConfig] = None,
                        max_model_len: int = 4096, tp: Optional[TPContext] = None, capture: bool = True,
                        dtype=torch.bfloat16, **arch_overrides):
        """A local HF-format checkpoint directory (config.json + *.safetensors)."""
        from src.models.loader import arch_from_hf_config, load_checkpoint

        arch = arch_from_hf_config(path, **arch_overrides)
        cfg = cfg or EngineConfig()
        model = CausalLM(arch, device, dtype=dtype, tp=tp, max_position=max(max_model_len, 16))
        load_checkpoint(model, path)
        eng = cls(model, cfg, max_model_len)
        if capture:
            eng.runner.capture_graphs()
        return eng

    # ------------------------------------------------------------ requests
    def add_request(self, request_id: str, prompt_ids: List[int], sampling: SamplingParams,
                    on_finish: Optional[Callable[[Sequence], None]] = None, user_data=None,
                    export_kv: bool = False,
                    on_token: Optional[Callable[[Sequence, int], None]] = None) -> Sequence:
        if request_id in self.seqs:
            raise ValueError(f"duplicate request id {request_id}")
        if len(prompt_ids) + sampling.max_tokens > self.max_model_len:
            raise ValueError(f"prompt + max_tokens exceeds max_model_len={self.max_model_len}")
        if prompt_ids and (min(prompt_ids) < 0 or max(prompt_ids) >= self.arch.vocab_size):
            # an out-of-range id would be an out-of-bounds embedding read on the GPU
            raise ValueError(f"prompt token id outside [0, {self.arch.vocab_size})")
        seq = Sequence(request_id, list(prompt_ids), dataclasses.replace(sampling), on_finish=on_finish,
                       user_data=user_data, on_token=on_token)
        if export_kv:  # disaggregated prefill: stop after the first token and hand the prompt KV over
            seq.sampling.max_tokens = 1
            seq.export_kv = True  # type: ignore[attr-defined]
        self.seqs[request_id] = seq
        if self.scheduler.running:
            self._dec_arrivals.append(time.perf_counter())
        self.scheduler.add(seq)
        self.stats["prompt_tokens"] += len(prompt_ids)
        return seq

    def add_imported(self, packet, sampling: SamplingParams,
                     on_finish: Optional[Callable[[Sequence], None]] = None) -> Sequence:
        """Resume a sequence whose prompt KV was computed by a prefill worker:
        allocate blocks, scatter the shipped KV into them, join the decode batch."""
        try:
            return self._add_imported(packet, sampling, on_finish)
        finally:
            # the packet's buffer (e.g. an IPC landing-zone slot) is free once the scatter queued above
            # has run: hand the importer an event recorded behind it (never a host sync)
            if getattr(packet, "on_imported", None) is not None:
                ev = None
                if packet.kv.is_cuda:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(self.device))
                packet.on_imported(ev)

    def _add_imported(self, packet, sampling: SamplingParams, on_finish) -> Sequence:
        from src.parallel.kv_transfer import import_blocks

        if packet.block_size != self.cfg.block_size:
            raise ValueError("block size mismatch between prefill and decode workers")
        self._last_import = time.perf_counter()
        seq = Sequence(packet.request_id, list(packet.prompt_ids), dataclasses.replace(sampling),
                       on_finish=on_finish, imported_kv=True)
        seq.output_ids = [int(packet.first_token)]
        seq.first_token_time = time.perf_counter()
        if packet.ttft_ms is not None:
            seq.arrival = seq.first_token_time - packet.ttft_ms / 1e3
        if len(seq) + sampling.max_tokens > self.max_model_len + 1:
            raise ValueError("imported sequence exceeds max_model_len")
        self.blocks.allocate(seq)
        nb = self.blocks.blocks_needed(seq.prompt_len)
        if packet.kv.shape[0] != nb:
            self.blocks.free(seq)
            raise ValueError(f"packet has {packet.kv.shape[0]} blocks, prompt needs {nb}")
        if getattr(packet, "ready", None) is not None:  # shipped on a transfer stream
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(packet.ready)
            packet.kv.record_stream(cur)
        import_blocks(self.pool.planes(), seq.block_table[:nb], packet.kv)
        seq.num_computed = seq.prompt_len
        self.seqs[seq.request_id] = seq
        self.stats["prompt_tokens"] += seq.prompt_len
        if len(seq.output_ids) >= seq.sampling.max_tokens:
            seq.status = SeqStatus.RUNNING
            self.scheduler.running.append(seq)
            self.scheduler.finish(seq, "length")
            self._complete(seq)
            return seq
        seq.status = SeqStatus.RUNNING
        self.scheduler.running.append(seq)
        return seq

    def abort(self, request_id: str) -> None:
        seq = self.scheduler.abort(request_id)
        if seq is not None:
            self._complete(seq)

    def has_work(self) -> bool:
        return self.scheduler.has_work() or self.runner.inflight is not None

    # ----------------------------------------------------------------- step
    def step(self) -> List[Sequence]:
        """One engine iteration. Returns the sequences that finished in it."""
        finished: List[Sequence] = []
        if self.runner.inflight is not None:
            # a decode window is queued on the GPU: queue the next one behind it when the batch is
            # unchanged (nothing waiting, nobody finishing by length), then apply its tokens while the
            # GPU runs on; otherwise apply them and schedule as usual
            seqs, pending = self.runner.inflight_batch()
            t0 = time.perf_counter()
            toks_k = self.runner.decode_continue(self._continuation_window(seqs, pending))
            now = time.perf_counter()
            self.stats["decode_time"] += now - t0
            self._apply_window(seqs, toks_k, finished)
            if self.runner.inflight is not None:
                self.stats["queued_windows"] = self.stats.get("queued_windows", 0) + 1
                self.stats["steps"] += 1
                return finished
        out: SchedulerOutput = self.scheduler.schedule()
        for s in out.preempted:
            if s.status == SeqStatus.FINISHED:  # rejected at admission
                s.finish_time = time.perf_counter()
                finished.append(s)
                self._complete(s)
        if out.swap_out or out.swap_in:
            self._run_swaps(out)
        if out.empty:
            return finished
        t0 = time.perf_counter()
        now = t0
        if out.prefill:
            # a prefill step, or a mixed step: the decode rows as 1-token chunks in the same ragged batch
            chunks = out.chunks() if out.decode else out.prefill
            exporter = self._start_export(chunks)
            try:
                toks = (self.runner.prefill(chunks) if exporter is None
                        else self.runner.prefill(chunks, kv_hook=exporter.on_layer))
            finally:
                # even when the forward fails: every slot the export took gets its completion event (a revoke then
                # releases it behind the queued gathers instead of polling until the TTL) and the compute stream
                # waits for those gathers before any later kernel can reuse the exported blocks
                if exporter is not None:
                    self._finish_export_safely(exporter)
            now = time.perf_counter()
            self.stats["mixed_time" if out.decode else "prefill_time"] = \
                self.stats.get("mixed_time" if out.decode else "prefill_time", 0.0) + now - t0
            ntok = sum(c.length for c in chunks if not c.decode)
            if ntok and not out.decode:
                per = (now - t0) / ntok
                self._pf_tok_est = per if not self._pf_tok_est else 0.8 * self._pf_tok_est + 0.2 * per
            for c, tok in zip(chunks, toks):
                seq = c.seq
                if c.decode:
                    if seq.status == SeqStatus.FINISHED:
                        continue
                    seq.num_computed += 1
                    self._append(seq, tok, finished)
                    continue
                seq.num_computed = c.start + c.length
                if tok is None:
                    continue
                self.blocks.register_prompt_blocks(seq)
                self.stats["prefix_hit_tokens"] += seq.num_prefix_hit
                if seq.first_token_time is None:
                    seq.first_token_time = now
                self._append(seq, tok, finished)
        else:
            k = self._decode_window(out.decode)
            if k > 1:
                toks_k = self.runner.decode_multi(out.decode, k, self._continuation_window(out.decode, k))
                if self.runner.inflight is not None:
                    self.stats["queued_windows"] = self.stats.get("queued_windows", 0) + 1
            else:
                toks_k = [self.runner.decode(out.decode)]
            now = time.perf_counter()
            self.stats["decode_time"] += now - t0
            self._step_est = 0.8 * self._step_est + 0.2 * (now - t0) / max(1, len(toks_k))
            self._apply_window(out.decode, toks_k, finished)
        self.stats["steps"] += 1
        if self.cfg.kv_block_ttl_s:
            self.blocks.evict_expired()
        self._update_load_snapshot()
        return finished

    def _update_load_snapshot(self) -> None:
        """The engine state a load balancer scores this worker by (src/load_balancer.py, least_latency), rebuilt
        by the engine thread after each step and swapped in whole (readers on other threads never see a
        half-built dict): sequences running / waiting, prompt tokens not yet prefilled, the batch cap, KV pool
        occupancy, and the EWMA decode step time and prefill time per prompt token."""
        sch = self.scheduler
        wt = 0
        for q in (sch.waiting, sch.running):
            for sq in q:
                if sq.num_computed < sq.prompt_len:
                    wt += sq.prompt_len - sq.num_computed
        self.load_snapshot = {"running": len(sch.running), "waiting": len(sch.waiting) + len(sch.swapped),
                              "waiting_prompt_tokens": wt, "max_num_seqs": self.cfg.max_num_seqs,
                              "kv_used_frac": round(self.blocks.usage(), 4),
                              "step_ms": round(self._step_est * 1e3, 4),
                              "prefill_us_per_token": round(self._pf_tok_est * 1e6, 3)}

    def _start_export(self, chunks):
        """Disaggregated prefill: the prompts that complete in this step and export their KV get their packets
        now (a reserved landing-zone slot — taken under its lock, see ExportSlot — or a staging tensor), and a
        LayerGroupExporter copies each group of layers into them while the rest of the forward runs. None when
        nothing exports (or off the GPU, under TP, or with cfg.kv_export_overlap off: the export then gathers
        everything after the step, in _append)."""
        from src.parallel.kv_transfer import LayerGroupExporter, packet_shape

        if self.device.type != "cuda" or not self.cfg.kv_export_overlap:
            return None
        if getattr(self.model, "tp", None) is not None and self.model.tp.enabled:
            return None
        planes = self.pool.planes()
        targets = []
        for c in chunks:
            seq = c.seq
            if c.decode or not c.completes_prompt or not getattr(seq, "export_kv", False):
                continue
            nb = self.blocks.blocks_needed(seq.prompt_len)
            ud = seq.user_data if isinstance(seq.user_data, dict) else {}
            slot = ud.get("export_slot")

            def dest(dst, nb=nb):
                buf = dst if dst is not None else torch.empty(packet_shape(planes, nb), dtype=planes.dtype,
                                                              device=planes.device)
                return buf, None
            buf, _ = slot.gather(dest) if slot is not None else dest(None)
            seq.kv_export = buf  # type: ignore[attr-defined]
            seq._export_slot_taken = slot if (slot is not None and slot.state == "taken") else None  # type: ignore
            targets.append((seq, list(seq.block_table[:nb]), buf))
        if not targets:
            return None
        ex = LayerGroupExporter(planes, self.arch.num_layers, [(ids, buf) for _, ids, buf in targets],
                                group=self.cfg.kv_export_group)
        ex.seqs = [s for s, _, _ in targets]
        return ex

    def _finish_export(self, ex) -> None:
        # the sender polls the completion event, then signals by RPC (an IPC completion event the decode worker's
        # stream waits on measured slower: 49.01 vs 49.55 req/s, profiles/disagg_r4_ipc_event_ab.jsonl)
        ev = ex.finish()
        for seq in ex.seqs:
            seq.kv_export_ready = ev  # type: ignore[attr-defined]
            slot = getattr(seq, "_export_slot_taken", None)
            if slot is not None:
                slot.set_event(ev)
        self.stats["overlapped_exports"] = self.stats.get("overlapped_exports", 0) + len(ex.seqs)

    def _finish_export_safely(self, ex) -> None:
        import sys

        if sys.exc_info()[0] is None:
            self._finish_export(ex)
            return
        try:  # the forward already raised: its exception is the one that propagates
            self._finish_export(ex)
        except Exception:  # noqa: BLE001
            logger.exception("finishing the KV export after a failed prefill step")

    def _run_swaps(self, out: SchedulerOutput) -> None:
        """Queue the step's KV swaps on the compute stream ahead of its forward: swap-outs pack
        the victim's blocks (move_blocks kernel) and copy them to pinned host memory without a
        host sync; swap-ins copy back and scatter into the freshly allocated blocks. Stream
        order makes the gathers read before any later kernel reuses the freed blocks."""
        from src.parallel.kv_transfer import export_blocks, import_blocks

        planes = self.pool.planes()
        # swap-ins first: a sequence resumed and (as a last resort) preempted again in the same step
        # must have its host KV scattered back before the swap-out gathers those blocks
        for seq, ids in out.swap_in:
            import_blocks(planes, ids, seq.swap_buf)
            seq.swap_buf = None
        for seq, ids in out.swap_out:
            buf = export_blocks(planes, ids)
            if buf.is_cuda:
                host = torch.empty(buf.shape, dtype=buf.dtype, pin_memory=True)
                host.copy_(buf, non_blocking=True)
                buf = host
            seq.swap_buf = buf
            self.stats["swap_out_bytes"] = self.stats.get("swap_out_bytes", 0) + buf.numel() * buf.element_size()

    def _apply_window(self, seqs: List[Sequence], toks_k: List[List[int]], finished: List[Sequence]) -> None:
        for toks in toks_k:
            for seq, tok in zip(seqs, toks):
                if seq.status == SeqStatus.FINISHED:  # stopped earlier in the window (or aborted): discard
                    continue
                seq.num_computed += 1
                self._append(seq, tok, finished)
        self.stats["decode_windows"] = self.stats.get("decode_windows", 0) + 1

    def _continuation_window(self, seqs: List[Sequence], pending: int) -> int:
        """Steps of a window to queue behind one of `pending` steps not yet applied (0: none). Only
        while the batch cannot change at the boundary: nothing waiting or swapped, every running
        sequence in the batch, none reaching max_tokens / the context limit within the queued
        window, and KV slots for both windows reserved now. An EOS inside the queued window only
        wastes the continuation's rows for that sequence (its tokens are discarded)."""
        if not self.cfg.async_decode or not getattr(self.runner, "supports_multistep", False):
            return 0
        sch = self.scheduler
        if sch.waiting or sch.swapped or len(sch.running) != len(seqs) or self._importing():
            return 0
        ids = {id(s) for s in seqs}
        if any(id(s) not in ids or s.status != SeqStatus.RUNNING or s.in_prefill for s in sch.running):
            return 0
        k = min(int(self.cfg.decode_window), self._arrival_cap(continuation=True),
                min(s.sampling.max_tokens - len(s.output_ids) - pending for s in seqs),
                min(self.max_model_len - (len(s) + pending) + 1 for s in seqs))
        if k <= 1:
            return 0
        for s in seqs:
            if not self.blocks.ensure_slots(s, len(s) + pending + k - 1):
                return 0
        return k

    def _recent_arrivals(self) -> List[float]:
        if self._arrival_lookback_s <= 0 or len(self._dec_arrivals) < 2:
            return []
        now = time.perf_counter()
        return [t for t in self._dec_arrivals if now - t < self._arrival_lookback_s]

    def _arrival_cap(self, continuation: bool = False) -> int:
        """While prompts keep arriving during decode (two or more in the lookback), no continuation window is
        queued behind the running one: a new prompt then waits for the rest of ONE window. (Shortening the
        windows to half the arrival gap instead gave TTFT p50 24 ms but TPOT +5 %, e2e +3 %: not kept.)"""
        if len(self._recent_arrivals()) < 2:
            return 1 << 30
        return 0 if continuation else 1 << 30

    def _importing(self) -> bool:
        """A burst of imported (disaggregated) prompts is still arriving."""
        return time.perf_counter() - self._last_import < self._import_settle_s

    def _decode_window(self, seqs: List[Sequence]) -> int:
        """How many decode steps to run before the host looks again: 1 while requests wait for
        admission (they must not sit behind a window), otherwise up to cfg.decode_window, no
        further than the longest remaining generation and the context limit, and only if KV
        slots for the whole window can be reserved now."""
        kmax = int(getattr(self.cfg, "decode_window", 1))
        if kmax <= 1 or not getattr(self.runner, "supports_multistep", False) or self._importing():
            return 1
        if self.scheduler.waiting:
            # prompts held for a larger prefill step (Scheduler._defer_prefill): a window that ends by
            # their deadline; otherwise they must not sit behind a window
            dl = self.scheduler.defer_deadline
            if dl is None:
                return 1
            kmax = min(kmax, int((dl - time.perf_counter()) / max(self._step_est, 1e-4)))
        k = min(kmax, self._arrival_cap(), max(s.sampling.max_tokens - len(s.output_ids) for s in seqs),
                min(self.max_model_len - len(s) + 1 for s in seqs))
        if k <= 1:
            return 1
        for s in seqs:
            if not self.blocks.ensure_slots(s, len(s) + k - 1):
                return 1
        return k

    def _append(self, seq: Sequence, tok: int, finished: List[Sequence]) -> None:
        seq.output_ids.append(int(tok))
        self.stats["generated_tokens"] += 1
        if seq.on_token is not None:
            seq.on_token(seq, int(tok))
        sp = seq.sampling
        reason = None
        if not sp.ignore_eos and self.eos_token_id is not None and tok == self.eos_token_id:
            reason = "stop"
        elif tok in sp.stop_token_ids:
            reason = "stop"
        elif len(seq.output_ids) >= sp.max_tokens:
            reason = "length"
        elif len(seq) >= self.max_model_len:
            reason = "length"
        if reason:
            if getattr(seq, "export_kv", False) and getattr(seq, "kv_export", None) is None:
                from src.parallel.kv_transfer import export_blocks

                nb = self.blocks.blocks_needed(seq.prompt_len)
                planes, ids = self.pool.planes(), seq.block_table[:nb]

                def gather(dst):
                    buf = export_blocks(planes, ids, out=dst)
                    ev = None
                    if buf.is_cuda:  # consumers wait on this instead of a host sync
                        ev = torch.cuda.Event()
                        ev.record()
                    return buf, ev

                # export_slot: a slot of the decode worker's landing zone reserved before the prompt ran (the
                # gather writes straight into it, unless the reservation is past its deadline or revoked);
                # else a local staging tensor
                ud = seq.user_data if isinstance(seq.user_data, dict) else {}
                slot = ud.get("export_slot")
                buf, ev = slot.gather(gather) if slot is not None else gather(None)
                seq.kv_export = buf  # type: ignore[attr-defined]
                if ev is not None:
                    seq.kv_export_ready = ev  # type: ignore[attr-defined]
            self.scheduler.finish(seq, reason)
            finished.append(seq)
            self._complete(seq)

    def _complete(self, seq: Sequence) -> None:
        self.seqs.pop(seq.request_id, None)
        self.stats["finished"] += 1
        prev = getattr(seq, "_preempted_outputs", None)
        if prev:
            seq.output_ids = prev + seq.output_ids
            seq.prompt_ids = seq.prompt_ids[: len(seq.prompt_ids) - len(prev)]
            seq._preempted_outputs = []  # type: ignore[attr-defined]
        if seq.on_finish is not None:
            seq.on_finish(seq)

    # ------------------------------------------------------------- helpers
    def generate(self, prompts: List[List[int]], sampling: SamplingParams) -> List[List[int]]:
        """Offline batch generation (blocking)."""
        res: Dict[str, List[int]] = {}
        for i, p in enumerate(prompts):
            self.add_request(f"gen-{i}-{time.monotonic_ns()}", p, sampling,
                             on_finish=lambda s, i=i: res.__setitem__(i, list(s.output_ids)))
        while self.has_work():
            self.step()
        return [res[i] for i in range(len(prompts))]

    def get_stats(self) -> dict:
        s = dict(self.stats)
        s.update(self.scheduler.stats())
        s["kv"] = self.blocks.stats()
        s["kv_pool_gib"] = self.pool.nbytes / 2**30
        s["graphs"] = list(self.runner.graph_sizes)
        s["decode_weight_layout"] = self.decode_weight_layout
        return s
