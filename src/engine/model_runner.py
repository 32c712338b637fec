"""
Model runner: turns a scheduled step into GPU work on one HIP stream.

* Step inputs are assembled by the native step builder
  (``csrc/runtime/step_builder.h``) straight into pinned host buffers and
  shipped with one async H2D copy per buffer.
* Prefill steps run eagerly (ragged shapes; their GEMMs dominate anyway).
* Decode steps replay a **hipGraph** captured per padded batch size
  (``EngineConfig.graph_batch_sizes``): embedding → 32 layers of
  norm/GEMM/RoPE+KV-write/paged-attention → LM head → sampling is one graph
  launch, so host launch overhead (≈10 launches × 32 layers) disappears.
  The graph reads everything from static buffers; the decode attention grid
  is sized for ``max_model_len`` and idle workgroups exit immediately.
* Only the token ids (8 B per sequence) come back to the host each step.
"""

from __future__ import annotations

import bisect
import logging
from typing import Dict, List, Optional, Sequence as Seq

import torch

from src import ops
from src.config import EngineConfig
from src.engine.block_manager import native_runtime
from src.engine.scheduler import PrefillChunk
from src.engine.sequence import Sequence
from src.models.llama import AttnMetadata, CausalLM

logger = logging.getLogger(__name__)


class KVPool:
    """One HBM tensor for the whole KV cache:
    [layers, 2 (K,V), num_blocks, kv_heads, block_size, head_dim] (bf16)."""

    def __init__(self, num_layers: int, num_blocks: int, kv_heads: int, block_size: int, head_dim: int, device,
                 dtype=torch.bfloat16):
        self.shape = (num_layers, 2, num_blocks, kv_heads, block_size, head_dim)
        # zeroed once: a padded graph row reads block 0 before anything was written there, and
        # uninitialised bf16 can hold NaN bit patterns
        self.tensor = torch.zeros(self.shape, dtype=dtype, device=device)
        self.num_blocks = num_blocks
        self.block_size = block_size

    @property
    def nbytes(self) -> int:
        return self.tensor.numel() * self.tensor.element_size()

    def planes(self) -> torch.Tensor:
        """[layers*2, num_blocks, ...] view used by the block movers."""
        s = self.shape
        return self.tensor.view(s[0] * s[1], s[2], s[3], s[4], s[5])

    @staticmethod
    def bytes_per_block(num_layers: int, kv_heads: int, block_size: int, head_dim: int, dtype_bytes: int = 2) -> int:
        return num_layers * 2 * kv_heads * block_size * head_dim * dtype_bytes


class ModelRunner:
    mirrors_windows = False  # see supports_multistep

    def __init__(self, model: CausalLM, pool: KVPool, cfg: EngineConfig, max_model_len: int):
        self.model = model
        self.pool = pool
        self.cfg = cfg
        self.device = model.device
        # prefill's last layer only for the sampled rows (CausalLM._last_layer_kept_rows)
        self.prune_last = True
        self.is_cuda = self.device.type == "cuda"
        self.bs = pool.block_size
        self.max_model_len = max_model_len
        self.bt_width = (max_model_len + self.bs - 1) // self.bs
        self.rt = native_runtime()
        self.max_seqs = cfg.max_num_seqs
        self.max_tokens = max(cfg.max_num_batched_tokens, self.max_seqs)
        pin = self.is_cuda
        i64, i32 = torch.int64, torch.int32
        # pinned host staging
        self.h_ids = torch.zeros(self.max_tokens, dtype=i64, pin_memory=pin)
        self.h_pos = torch.zeros(self.max_tokens, dtype=i64, pin_memory=pin)
        self.h_slots = torch.zeros(self.max_tokens, dtype=i64, pin_memory=pin)
        self.h_cu = torch.zeros(self.max_seqs + 1, dtype=i32, pin_memory=pin)
        self.h_ctx = torch.zeros(self.max_seqs, dtype=i32, pin_memory=pin)
        self.h_bt = torch.zeros(self.max_seqs, self.bt_width, dtype=i32, pin_memory=pin)
        self.h_last = torch.zeros(self.max_seqs, dtype=i64, pin_memory=pin)
        self.h_temp = torch.zeros(self.max_seqs, dtype=torch.float32, pin_memory=pin)
        self.h_topk = torch.zeros(self.max_seqs, dtype=i32, pin_memory=pin)
        self.h_topp = torch.ones(self.max_seqs, dtype=torch.float32, pin_memory=pin)
        self.h_seed = torch.zeros(self.max_seqs, dtype=i64, pin_memory=pin)
        self.h_step = torch.zeros(self.max_seqs, dtype=i64, pin_memory=pin)
        self.h_out = torch.zeros(self.max_seqs, dtype=i64, pin_memory=pin)
        self.k_max = max(1, int(getattr(cfg, "decode_window", 1)))
        # two halves of k_max rows: a window's tokens land in one half while the next (continuation)
        # window, already queued behind it, writes the other
        self.h_tokens = torch.zeros(2 * self.k_max, self.max_seqs, dtype=i64, pin_memory=pin)
        # continuation-window staging (block tables + first-step slots), double-buffered by parity: a
        # set is rewritten only after the window that read it has been waited for
        self.h_cbt = [torch.zeros(self.max_seqs, self.bt_width, dtype=i32, pin_memory=pin) for _ in range(2)]
        self.h_cslots = [torch.zeros(self.max_seqs, dtype=i64, pin_memory=pin) for _ in range(2)]
        self.h_cscratch = (torch.zeros(self.max_seqs, dtype=i64), torch.zeros(self.max_seqs, dtype=i32))
        self._cpar = 0
        self.inflight: Optional[Dict[str, object]] = None  # a queued window whose tokens are not yet read
        self.h_ctl = torch.zeros(2, dtype=i32, pin_memory=pin)   # [window step counter, real rows]
        # numpy views over the pinned buffers (zero-copy) for cheap bulk writes
        self.n_ids, self.n_temp, self.n_topk = self.h_ids.numpy(), self.h_temp.numpy(), self.h_topk.numpy()
        self.n_topp, self.n_seed, self.n_step = self.h_topp.numpy(), self.h_seed.numpy(), self.h_step.numpy()
        self._samp_key = None
        self._samp_dirty = False
        dev = self.device
        # device-side static buffers (graph inputs)
        self.d_ids = torch.zeros(self.max_tokens, dtype=i64, device=dev)
        self.d_pos = torch.zeros(self.max_tokens, dtype=i64, device=dev)
        self.d_slots = torch.zeros(self.max_tokens, dtype=i64, device=dev)
        self.d_cu = torch.zeros(self.max_seqs + 1, dtype=i32, device=dev)
        self.d_ctx = torch.ones(self.max_seqs, dtype=i32, device=dev)
        self.d_bt = torch.zeros(self.max_seqs, self.bt_width, dtype=i32, device=dev)
        self.d_last = torch.zeros(self.max_seqs, dtype=i64, device=dev)
        self.d_temp = torch.zeros(self.max_seqs, dtype=torch.float32, device=dev)
        self.d_topk = torch.zeros(self.max_seqs, dtype=i32, device=dev)
        self.d_topp = torch.ones(self.max_seqs, dtype=torch.float32, device=dev)
        self.d_seed = torch.zeros(self.max_seqs, dtype=i64, device=dev)
        self.d_step = torch.zeros(self.max_seqs, dtype=i64, device=dev)
        self.d_out = torch.zeros(self.max_seqs, dtype=i64, device=dev)
        # split greedy argmax scratch (ops.sample): per-slice (max, index) and per-row tickets, re-armed in-kernel
        self.d_samp = (torch.zeros(self.max_seqs * 32, dtype=torch.int32, device=dev),
                       torch.zeros(self.max_seqs, dtype=torch.int32, device=dev))
        self.d_tokens = torch.zeros(2 * self.k_max, self.max_seqs, dtype=i64, device=dev)
        self.d_ctl = torch.zeros(2, dtype=i32, device=dev)
        self.d_adv_ticket = torch.zeros(1, dtype=i32, device=dev)  # sample_advance's row ticket (re-armed in-kernel)
        if self.is_cuda:
            maxp = ops.decode_partials(max_model_len)
            hq = model.hq
            self.part_o = torch.empty(self.max_seqs * hq * maxp * 128, dtype=torch.float32, device=dev)
            self.part_ml = torch.empty(self.max_seqs * hq * maxp * 2, dtype=torch.float32, device=dev)
            self.attn_cnt = torch.zeros(self.max_seqs * model.hkv, dtype=i32, device=dev)
            self.dec_scratch = (model.alloc_decode_scratch(self.max_seqs) if hasattr(model, "alloc_decode_scratch")
                                else None)
            # the LM head's per-column-tile greedy candidates (CausalLM.compute_logits(argmax_parts=...)): a greedy
            # row's argmax reduces those instead of re-reading its 128K logits (decode steps of <= 128 rows)
            parts = model.lm_head_argmax_parts() if hasattr(model, "lm_head_argmax_parts") else 0
            self.d_lmpart = torch.zeros(self.max_seqs, parts, 2, dtype=i32, device=dev) if parts else None
        else:
            self.part_o = self.part_ml = self.attn_cnt = self.dec_scratch = self.d_lmpart = None
        self.supports_swap = type(self)._sync_step is ModelRunner._sync_step
        # a runner whose steps are mirrored by other ranks (tensor parallelism) must mirror whole windows too:
        # it declares that with mirrors_windows (TPModelRunner sends one message per window, not per step)
        self.supports_multistep = self.is_cuda and self.k_max > 1 and (
            type(self)._sync_step is ModelRunner._sync_step or self.mirrors_windows)
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_sizes: List[int] = []
        self._graph_pool = None
        self.stream = torch.cuda.current_stream(dev) if self.is_cuda else None

    # ------------------------------------------------------------ helpers
    def _h2d(self, n_tok: int, n_seq: int, with_cu: bool) -> None:
        nb = self.is_cuda
        self.d_ids[:n_tok].copy_(self.h_ids[:n_tok], non_blocking=nb)
        self.d_pos[:n_tok].copy_(self.h_pos[:n_tok], non_blocking=nb)
        self.d_slots[:n_tok].copy_(self.h_slots[:n_tok], non_blocking=nb)
        self.d_ctx[:n_seq].copy_(self.h_ctx[:n_seq], non_blocking=nb)
        self.d_bt[:n_seq].copy_(self.h_bt[:n_seq], non_blocking=nb)
        if with_cu:
            self.d_cu[: n_seq + 1].copy_(self.h_cu[: n_seq + 1], non_blocking=nb)
            self.d_last[:n_seq].copy_(self.h_last[:n_seq], non_blocking=nb)

    def _fill_sampling(self, seqs: Seq[Sequence], n_pad: int) -> bool:
        """Write per-row sampling params; returns True when every row is greedy.
        Skips the H2D copies when the rows are all greedy (the kernel's greedy
        path ignores them) — the common decode case costs nothing here."""
        greedy = all(s.sampling.greedy for s in seqs)
        if greedy:
            key = ("greedy", n_pad)
            if self._samp_key == key:
                return True
            self.n_temp[:n_pad] = 0.0
            self.n_topk[:n_pad] = 0
            self.n_topp[:n_pad] = 1.0
            self._samp_key = key
        else:
            n = len(seqs)
            self.n_temp[:n] = [s.sampling.temperature for s in seqs]
            self.n_topk[:n] = [s.sampling.top_k for s in seqs]
            self.n_topp[:n] = [s.sampling.top_p for s in seqs]
            self.n_seed[:n] = [s.sampling.seed if s.sampling.seed is not None else s.seq_id for s in seqs]
            self.n_step[:n] = [len(s.output_ids) + len(getattr(s, "_preempted_outputs", ())) for s in seqs]
            self.n_temp[n:n_pad] = 0.0
            self.n_topk[n:n_pad] = 0
            self.n_topp[n:n_pad] = 1.0
            self._samp_key = None
        nb = self.is_cuda
        for h, d in ((self.h_temp, self.d_temp), (self.h_topk, self.d_topk), (self.h_topp, self.d_topp),
                     (self.h_seed, self.d_seed), (self.h_step, self.d_step)):
            d[:n_pad].copy_(h[:n_pad], non_blocking=nb)
        self._samp_dirty = True  # the device-side parameters changed since a TP leader last mirrored them
        return greedy

    def _sample(self, logits: torch.Tensor, n: int, greedy: bool, out: torch.Tensor) -> torch.Tensor:
        if greedy:
            return ops.sample(logits, out=out[:n], scratch=self.d_samp) if self.is_cuda else ops.sample(logits)
        args = (self.d_temp[:n], self.d_topk[:n], self.d_topp[:n], self.d_seed[:n], self.d_step[:n])
        return ops.sample(logits, *args, out=out[:n], scratch=self.d_samp) if self.is_cuda else ops.sample(logits, *args)

    def _to_host(self, ids: torch.Tensor, n: int) -> List[int]:
        if self.is_cuda:
            self.h_out[:n].copy_(ids[:n], non_blocking=True)
            self._queue_fault_readback()
            torch.cuda.current_stream(self.device).synchronize()
            self._raise_on_fault()
            return self.h_out[:n].tolist()
        return ids[:n].tolist()

    def _queue_fault_readback(self) -> None:
        """Queue device-side error words behind the step (read with the tokens, same sync). None on one GPU;
        the TP runner reads the one-shot collectives' sticky error word."""

    def _raise_on_fault(self) -> None:
        """Raise if an error word read by :meth:`_queue_fault_readback` is set."""

    # ------------------------------------------------------------ prefill
    KIND_STOP, KIND_PREFILL, KIND_DECODE, KIND_HEARTBEAT = 0, 1, 2, 3

    def idle_tick(self) -> None:
        """Called by the engine loop while it has no work (TP runners send heartbeats)."""

    def _sync_step(self, kind: int, a: int = 0, b: int = 0, c: int = 0, d: int = 0) -> None:
        """Hook for tensor parallelism: rank 0 publishes the step to followers
        (see :class:`src.parallel.tp_runner.TPModelRunner`). No-op at TP=1."""

    def _sync_window(self, n: int, pad: int, k: int) -> None:
        """Hook: rank 0 publishes a k-step decode window (its first step's inputs, already in the host staging
        buffers; the graph advances them on every rank). No-op at TP=1."""

    def _sync_continuation(self, par: int, pad: int, k: int, base: int) -> None:
        """Hook: rank 0 publishes a continuation window queued behind the running one (the re-sent block tables
        and first-step slots of staging set ``par``, the token-row base). No-op at TP=1."""

    @torch.inference_mode()
    def prefill(self, chunks: List[PrefillChunk], kv_hook=None) -> List[Optional[int]]:
        """Run one ragged prefill batch — or a mixed step, whose decode rows are 1-token chunks —
        and return the sampled token for every chunk that completes its prompt or decodes
        (None for partial prompt chunks)."""
        toks = [c.tokens() for c in chunks]
        starts = [c.start for c in chunks]
        tables = [c.seq.block_table for c in chunks]
        n = len(chunks)
        t = self.rt.build_prefill_inputs(toks, starts, tables, self.bs, self.h_ids.data_ptr(),
                                         self.h_pos.data_ptr(), self.h_slots.data_ptr(), self.h_cu.data_ptr(),
                                         self.h_ctx.data_ptr(), self.h_bt.data_ptr(), self.bt_width,
                                         self.h_last.data_ptr())
        done = [i for i, c in enumerate(chunks) if c.completes_prompt]
        nd = len(done)
        if nd and nd != n:
            nl = self.h_last.numpy()
            nl[:nd] = nl[done]
        greedy = self._fill_sampling([chunks[i].seq for i in done], nd) if nd else True
        self._h2d(t, n, with_cu=True)
        max_q = max(c.length for c in chunks)
        self._sync_step(self.KIND_PREFILL, t, n, max_q, nd)
        ids = self._exec_prefill(t, n, max_q, nd, greedy, kv_hook=kv_hook)
        res: List[Optional[int]] = [None] * n
        if nd:
            vals = self._to_host(ids, nd)
            for j, i in enumerate(done):
                res[i] = vals[j]
        elif self.is_cuda:
            self._queue_fault_readback()
            torch.cuda.current_stream(self.device).synchronize()
            self._raise_on_fault()
        return res

    def _exec_prefill(self, t: int, n: int, max_q: int, nd: int, greedy: bool, kv_hook=None) -> Optional[torch.Tensor]:
        # the last layer runs only for the sampled rows (CausalLM._last_layer_kept_rows; DIE_PRUNE_LAST=0: all)
        keep = self.d_last[:nd] if self.prune_last else None
        meta = AttnMetadata(is_prefill=True, slot_mapping=self.d_slots[:t], block_tables=self.d_bt[:n],
                            ctx_lens=self.d_ctx[:n], cu_q=self.d_cu[: n + 1], max_q_len=max_q, kv_hook=kv_hook,
                            keep_rows=keep)
        hidden = self.model.forward(self.d_ids[:t], self.d_pos[:t], meta, self.pool.tensor)
        if not nd:
            return None
        if hidden.shape[0] != nd:  # a path that computed every row (e.g. the slab path of small steps)
            hidden = hidden.index_select(0, self.d_last[:nd])
        logits = self.model.compute_logits(hidden)
        return self._sample(logits, nd, greedy, self.d_out)

    # ------------------------------------------------------------- decode
    def _fused_tail(self, n: int) -> bool:
        """Steps of n rows end in ONE launch that samples from the LM head's candidates, advances the inputs and
        gathers the next step's embedding rows (ops.sample_advance): then the step itself starts from them
        (AttnMetadata.pre_embedded) and the host writes them before the first step of a window (_pre_embed)."""
        return bool(self.supports_multistep and self.d_lmpart is not None and n <= ops.DECODE_GEMM_MAX_M
                    and self.model.lm_head_argmax_parts() == self.d_lmpart.shape[1]
                    and self.dec_scratch is not None and n <= self.dec_scratch["h_in"].shape[0])

    def _pre_embed(self, pad: int) -> None:
        if self._fused_tail(pad):
            sc = self.dec_scratch
            ops.embed_sumsq(self.d_ids[:pad], self.model.embed, sc["ssp0"], out=sc["h_in"][:pad])

    def _decode_forward(self, n: int) -> torch.Tensor:
        tail = self._fused_tail(n)
        meta = AttnMetadata(is_prefill=False, slot_mapping=self.d_slots[:n], block_tables=self.d_bt[:n],
                            ctx_lens=self.d_ctx[:n], max_ctx=self.max_model_len, part_o=self.part_o,
                            part_ml=self.part_ml, attn_cnt=self.attn_cnt, scratch=self.dec_scratch,
                            pre_embedded=tail)
        hidden = self.model.forward(self.d_ids[:n], self.d_pos[:n], meta, self.pool.tensor)
        amax = (self.d_lmpart if self.d_lmpart is not None and n <= ops.DECODE_GEMM_MAX_M
                and self.model.lm_head_argmax_parts() == self.d_lmpart.shape[1] else None)
        logits = self.model.compute_logits(hidden, argmax_parts=amax) if amax is not None else \
            self.model.compute_logits(hidden)
        if not self.is_cuda:
            return ops.sample(logits, self.d_temp[:n], self.d_topk[:n], self.d_topp[:n], self.d_seed[:n],
                              self.d_step[:n])
        if tail:
            # sampling from the LM head's candidates, the next step's input advance and its embedding rows in one launch
            sc = self.dec_scratch
            return ops.sample_advance(logits, self.d_temp[:n], self.d_topk[:n], self.d_topp[:n], self.d_seed[:n],
                                      self.d_step, self.d_out[:n], amax[:n], self.d_ids, self.d_pos, self.d_ctx,
                                      self.d_slots, self.d_bt, self.d_tokens, self.d_ctl[0:1], self.d_ctl[1:2],
                                      self.bs, self.d_adv_ticket,
                                      embed=(self.model.embed, sc["h_in"], sc["ssp0"].view(-1)))
        out = ops.sample(logits, self.d_temp[:n], self.d_topk[:n], self.d_topp[:n], self.d_seed[:n],
                         self.d_step[:n], out=self.d_out[:n], scratch=self.d_samp,
                         lm_part=amax[:n] if amax is not None else None)
        if self.supports_multistep:
            # next step's inputs from this step's samples, on the device (multi-step windows)
            ops.decode_advance(self.d_out, self.d_ids, self.d_pos, self.d_ctx, self.d_slots, self.d_bt, self.d_step,
                               self.d_tokens, self.d_ctl[0:1], self.d_ctl[1:2], n, self.bs)
        return out

    @torch.inference_mode()
    def capture_graphs(self) -> None:
        if not self.is_cuda or not self.cfg.use_cuda_graph:
            return
        sizes = sorted({min(b, self.max_seqs) for b in self.cfg.graph_batch_sizes} | {self.max_seqs})
        self._graph_pool = torch.cuda.graph_pool_handle()
        # warm up (hipBLASLt heuristics, kernel loads) outside capture
        for b in sizes:
            self.d_slots[:b].fill_(-1)
            self.d_ctx[:b].fill_(1)
            self._decode_forward(b)
        torch.cuda.synchronize(self.device)
        for b in reversed(sizes):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._graph_pool):
                self._decode_forward(b)
            self.graphs[b] = g
        torch.cuda.synchronize(self.device)
        self.graph_sizes = sizes
        logger.info("captured decode hipGraphs for batch sizes %s", sizes)

    def _pad_for(self, n: int) -> int:
        if self.graphs:
            k = bisect.bisect_left(self.graph_sizes, n)
            if k < len(self.graph_sizes):
                return self.graph_sizes[k]
        return n

    @torch.inference_mode()
    def decode(self, seqs: List[Sequence]) -> List[int]:
        n = len(seqs)
        pad = self._pad_for(n)
        self.n_ids[:n] = [s.last_token for s in seqs]
        self.n_ids[n:pad] = 0
        self.rt.build_decode_inputs([s.block_table for s in seqs], [len(s) for s in seqs], self.bs,
                                    self.h_pos.data_ptr(), self.h_slots.data_ptr(), self.h_ctx.data_ptr(),
                                    self.h_bt.data_ptr(), self.bt_width, pad)
        self._fill_sampling(seqs, pad)
        self._h2d(pad, pad, with_cu=False)
        self._pre_embed(pad)  # the step starts from these rows when its tail launch writes the next ones
        if self.supports_multistep:  # the graph's input advance must see this step's real rows
            self.h_ctl[0] = 0
            self.h_ctl[1] = n
            self.d_ctl.copy_(self.h_ctl, non_blocking=True)
        self._sync_step(self.KIND_DECODE, n, pad)
        ids = self._exec_decode(n, pad)
        return self._to_host(ids, n)

    @torch.inference_mode()
    def decode_multi(self, seqs: List[Sequence], k: int, k_next: int = 0) -> List[List[int]]:
        """k decode steps for the same batch in one host round trip: the step's hipGraph ends
        with a device-side input advance (sampled ids -> next ids, positions/context/step + 1,
        next slot from the block table), so the graph is replayed k times back to back and the
        k x n sampled tokens come back in one copy. The caller has reserved KV slots for the
        k positions. Falls back to single steps where no graph covers the batch.

        k_next > 1 (slots reserved for k + k_next positions): a continuation window of k_next
        steps is queued behind this one before the host waits, so the GPU runs it while the
        caller applies this window's tokens; :meth:`decode_continue` collects it."""
        n = len(seqs)
        pad = self._pad_for(n)
        g = self.graphs.get(pad)
        if k <= 1 or g is None or not self.supports_multistep:
            return [self.decode(seqs)]
        assert self.inflight is None, "a queued decode window must be collected first"
        k = min(k, self.k_max)
        self.n_ids[:n] = [s.last_token for s in seqs]
        self.n_ids[n:pad] = 0
        self.rt.build_decode_inputs([s.block_table for s in seqs], [len(s) for s in seqs], self.bs,
                                    self.h_pos.data_ptr(), self.h_slots.data_ptr(), self.h_ctx.data_ptr(),
                                    self.h_bt.data_ptr(), self.bt_width, pad)
        self._fill_sampling(seqs, pad)
        self._h2d(pad, pad, with_cu=False)
        self._pre_embed(pad)  # the step starts from these rows when its tail launch writes the next ones
        self.h_ctl[0] = 0
        self.h_ctl[1] = n
        self.d_ctl.copy_(self.h_ctl, non_blocking=True)
        self._sync_window(n, pad, k)
        for _ in range(k):
            g.replay()
        self.h_tokens[:k].copy_(self.d_tokens[:k], non_blocking=True)
        self._queue_fault_readback()
        if k_next > 1:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._queue_continuation(seqs, k, k_next, base=self.k_max)
            ev.synchronize()
        else:
            torch.cuda.current_stream(self.device).synchronize()
        self._raise_on_fault()
        return self.h_tokens[:k, :n].tolist()

    def _queue_continuation(self, seqs: List[Sequence], pending: int, k: int, base: int) -> None:
        """Queue k more decode steps for `seqs` behind a window of `pending` steps whose tokens the
        host has not applied yet (len(s) excludes them). Positions, context lengths and ids are
        already advanced on the device; the block tables (grown for the new positions) and the
        first step's slots (the queued window's last advance read the old tables) are re-sent."""
        n = len(seqs)
        pad = self._pad_for(n)
        k = min(k, self.k_max)
        par = self._cpar
        self._cpar ^= 1
        hbt, hsl = self.h_cbt[par], self.h_cslots[par]
        spos, sctx = self.h_cscratch
        self.rt.build_decode_inputs([s.block_table for s in seqs], [len(s) + pending for s in seqs], self.bs,
                                    spos.data_ptr(), hsl.data_ptr(), sctx.data_ptr(), hbt.data_ptr(),
                                    self.bt_width, pad)
        self.d_bt[:pad].copy_(hbt[:pad], non_blocking=True)
        self.d_slots[:pad].copy_(hsl[:pad], non_blocking=True)
        self.d_ctl[0:1].fill_(base)  # token rows [base, base + k)
        self._sync_continuation(par, pad, k, base)
        g = self.graphs[pad]
        for _ in range(k):
            g.replay()
        self.h_tokens[base:base + k].copy_(self.d_tokens[base:base + k], non_blocking=True)
        self._queue_fault_readback()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.inflight = {"seqs": list(seqs), "k": k, "base": base, "event": ev}

    def inflight_batch(self):
        """(sequences, steps) of the queued window, or None."""
        w = self.inflight
        return None if w is None else (w["seqs"], w["k"])

    @torch.inference_mode()
    def decode_continue(self, k_next: int = 0) -> List[List[int]]:
        """Collect the queued window's tokens ([k][n]); first, if k_next > 1 (the caller reserved
        the slots and the batch is unchanged), queue the next window behind it."""
        w = self.inflight
        assert w is not None
        self.inflight = None
        if k_next > 1:
            self._queue_continuation(w["seqs"], w["k"], k_next, base=self.k_max - w["base"])
        w["event"].synchronize()
        self._raise_on_fault()
        b, k, n = w["base"], w["k"], len(w["seqs"])
        return self.h_tokens[b:b + k, :n].tolist()

    def _exec_decode(self, n: int, pad: int) -> torch.Tensor:
        g = self.graphs.get(pad)
        if g is not None:
            g.replay()
            return self.d_out
        return self._decode_forward(n)
