"""
Llama-3 / Mixtral decoder on PyTorch-ROCm + the gfx950 kernels of :mod:`src.ops`.

Per decoder layer (T = tokens of the step):

    x   = fused_add_rms_norm(h, residual, ln1)          HIP  (residual += h in place)
    qkv = x @ Wqkv^T                                    hipBLASLt   [T, (hq+2hkv)*128]
    rope_and_cache(k rotated, k/v → paged HBM blocks; prefill q is rotated by the attention Q load)   HIP
    a   = attn_prefill | attn_decode (paged, GQA)       HIP  (MFMA)
    o   = a @ Wo^T   (+ all_reduce over RCCL if TP)     hipBLASLt
    x   = fused_add_rms_norm(o, residual, ln2)          HIP
    Llama:   d = silu_and_mul(x @ Wgu^T) @ Wd^T          hipBLASLt + HIP
    Mixtral: d = moe_forward(x, router)                  HIP routing + expert-streaming grouped GEMM
    (+ all_reduce if TP)

Weights are stored pre-fused ([q|k|v] and [gate|up]) so each projection is one
GEMM. Only the last token of each prefill sequence reaches the LM head.
The same module runs CPU tensors through :mod:`src.ops.reference` for tests.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import torch
import torch.nn.functional as F

from src import ops
from src.models.presets import ArchConfig
from src.ops.reference import rope_cos_sin
from src.parallel.tp import TPContext


@dataclass
class AttnMetadata:
    """Everything the attention kernels need for one step (device tensors)."""

    is_prefill: bool
    slot_mapping: torch.Tensor      # [T] int64, -1 = do not write KV
    block_tables: torch.Tensor      # [S, W] int32
    ctx_lens: torch.Tensor          # [S] int32 (KV length after this step)
    cu_q: Optional[torch.Tensor] = None    # [S+1] int32 (prefill)
    max_q_len: int = 1
    max_ctx: int = 0                # decode grid bound (static under hipGraph)
    part_o: Optional[torch.Tensor] = None
    part_ml: Optional[torch.Tensor] = None
    attn_cnt: Optional[torch.Tensor] = None  # decode attention merge tickets (int32, zeroed once)
    scratch: Optional[dict] = None  # fused decode path buffers (CausalLM.alloc_decode_scratch)
    kv_hook: Optional[Callable[[int], None]] = None  # prefill: called once layer i's KV writes are queued
    # prefill: the only rows whose final hidden state is used (each sampled chunk's last token, [n] int64): the
    # last layer computes its KV for every token but attention / o / MLP / final norm only for these rows, and
    # forward() returns [n, H] in this order (None: every row)
    keep_rows: Optional[torch.Tensor] = None
    # decode (fused path): the step's embedding rows and first-norm statistics are already in scratch["h_in"] /
    # scratch["ssp0"] (written by the previous step's sampling launch, or by the runner before a window)
    pre_embedded: bool = False


class LayerWeights:
    # tiled: decode-GEMM tile-order copies {(projection, wr, kc): tensor} (CausalLM.pack_decode_weights)
    __slots__ = ("ln1", "ln2", "qkv", "o", "gate_up", "down", "router", "w13", "w2", "tiled")

    def __init__(self):
        for s in self.__slots__:
            setattr(self, s, None)
        self.tiled = {}


# LDS staging area of the fused decode attention's prologue (csrc/kernels/attention.hip V3_MERGE)
V3_MERGE_BYTES = 27 * 1024

class CausalLM:
    """A TP-sharded decoder-only LM (no nn.Module overhead on the hot path)."""

    def __init__(self, arch: ArchConfig, device, dtype=torch.bfloat16, tp: Optional[TPContext] = None,
                 seed: int = 0, init_std: float = 0.02, max_position: Optional[int] = None,
                 full_init: bool = False, moe_parallel: str = "tp", sequence_parallel: bool = False):
        """``full_init=True`` draws every weight at full (unsharded) size from a
        rank-independent generator and slices this rank's shard — identical to
        the TP=1 model, used by the TP equivalence tests. The default draws
        only the local shard (never materialises a 70B tensor).

        ``moe_parallel`` (MoE models under TP): ``"tp"`` splits every expert's FFN dimension over
        the ranks; ``"ep"`` (expert parallelism) gives each rank whole experts
        ``[rank * E/tp, (rank + 1) * E/tp)`` — bigger per-expert GEMMs, no FFN-dim divisibility
        constraint. Attention stays tensor-parallel, so every rank holds every token: the routed
        assignments to remote experts are masked locally and the MoE's TP all-reduce is the combine
        (no all-to-all, see ops.expert_parallel_local).

        ``sequence_parallel`` (TP prefill): Megatron-SP — the residual stream and the norms are
        sharded over the ranks by token; each layer's two all-reduces become a reduce-scatter into
        the norm and an all-gather out of it (same bytes on the links, 1/W of the norm work and of
        the residual's memory). Decode steps (<= 32 rows) keep the all-reduce path."""
        self.arch = arch
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPContext()
        a, tpc = arch, self.tp
        self.hq = tpc.shard(a.num_heads)
        self.hkv = tpc.kv_heads(a.num_kv_heads)
        self.ep = bool(a.is_moe and tpc.enabled and moe_parallel == "ep")
        if moe_parallel not in ("tp", "ep"):
            raise ValueError(f"moe_parallel must be 'tp' or 'ep', got {moe_parallel!r}")
        if self.ep:
            self.experts_local = tpc.shard(a.num_experts)
            self.expert0 = tpc.rank * self.experts_local
            self.inter = a.intermediate_size  # whole experts per rank
        else:
            self.experts_local, self.expert0 = a.num_experts, 0
            self.inter = tpc.shard(a.intermediate_size)
        self.vocab_local = tpc.shard(a.vocab_size) if a.vocab_size % tpc.world_size == 0 else a.vocab_size
        self.vocab_parallel = self.vocab_local != a.vocab_size
        self.head_dim = a.head_dim
        self.scale = 1.0 / math.sqrt(a.head_dim)
        self.max_position = max_position or a.max_position
        self.full_init = full_init
        self.sequence_parallel = bool(sequence_parallel and self.tp.enabled)
        self.tiled_decode_weights = True  # decode GEMMs on tile-order copies (pack_decode_weights)
        self.lm_head_tile = None          # (wr, kc) once the LM head is re-laid in place in tile order
        self.prefill_gemm_residual = True  # TP=1 prefill: o / down add into the residual in the GEMM (beta = 1)
        self.layers: List[LayerWeights] = []
        self._init_random(seed, init_std)
        self.cos_sin = rope_cos_sin(self.max_position, a.head_dim, a.rope_theta, self.device, a.rope_scaling)

    # ------------------------------------------------------------------ init
    def _randn(self, *shape, std: float, gen) -> torch.Tensor:
        t = torch.empty(*shape, dtype=self.dtype, device=self.device)
        t.normal_(0.0, std, generator=gen)
        return t

    # TP slicing of full-size tensors (Megatron layout, see src/parallel/tp.py)
    def shard_qkv(self, full: torch.Tensor) -> torch.Tensor:
        a, r, d = self.arch, self.tp.rank, self.head_dim
        hq, hkv = self.hq, self.hkv
        kv_idx = (r * hkv) if a.num_kv_heads >= self.tp.world_size else r // (self.tp.world_size // a.num_kv_heads)
        q = full[r * hq * d:(r + 1) * hq * d]
        k0 = a.num_heads * d + kv_idx * d
        v0 = (a.num_heads + a.num_kv_heads) * d + kv_idx * d
        return torch.cat([q, full[k0:k0 + hkv * d], full[v0:v0 + hkv * d]], 0)

    def shard_cols(self, full: torch.Tensor, n_local: int) -> torch.Tensor:
        r = self.tp.rank
        return full[..., r * n_local:(r + 1) * n_local]

    def shard_gate_up(self, full: torch.Tensor) -> torch.Tensor:
        r, i = self.tp.rank, self.inter
        big = self.arch.intermediate_size
        g = full[..., r * i:(r + 1) * i, :]
        u = full[..., big + r * i:big + (r + 1) * i, :]
        return torch.cat([g, u], -2)

    def shard_rows(self, full: torch.Tensor, n_local: int) -> torch.Tensor:
        r = self.tp.rank
        return full[r * n_local:(r + 1) * n_local]

    def _param(self, local_shape, full_shape, shard, std, gen_local, gen_full):
        if self.full_init and self.tp.enabled:
            return shard(self._randn(*full_shape, std=std, gen=gen_full)).contiguous()
        return self._randn(*local_shape, std=std, gen=gen_full if not self.tp.enabled else gen_local)

    def _init_random(self, seed: int, std: float) -> None:
        a = self.arch
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed * 7919 + self.tp.rank)
        genf = torch.Generator(device=self.device)   # rank-independent stream
        genf.manual_seed(seed * 7919 + 104729)
        h, d, L = a.hidden_size, a.head_dim, a.num_layers
        ostd = std / math.sqrt(2 * L)
        # Embedding replicated on every rank: identical across ranks.
        gen_e = torch.Generator(device=self.device)
        gen_e.manual_seed(seed)
        self.embed = self._randn(a.vocab_size, h, std=1.0, gen=gen_e)
        nq, nkv, big = a.num_heads, a.num_kv_heads, a.intermediate_size
        for _ in range(L):
            lw = LayerWeights()
            lw.ln1 = torch.ones(h, dtype=self.dtype, device=self.device)
            lw.ln2 = torch.ones(h, dtype=self.dtype, device=self.device)
            lw.qkv = self._param(((self.hq + 2 * self.hkv) * d, h), ((nq + 2 * nkv) * d, h), self.shard_qkv,
                                 std, gen, genf)
            lw.o = self._param((h, self.hq * d), (h, nq * d), lambda t: self.shard_cols(t, self.hq * d), ostd,
                               gen, genf)
            if a.is_moe:
                lw.router = self._randn(a.num_experts, h, std=std, gen=gen_e)  # replicated router
                if self.ep:  # whole experts [expert0, expert0 + experts_local)
                    e0, el = self.expert0, self.experts_local
                    lw.w13 = self._param((el, 2 * big, h), (a.num_experts, 2 * big, h), lambda t: t[e0:e0 + el],
                                         std, gen, genf)
                    lw.w2 = self._param((el, h, big), (a.num_experts, h, big), lambda t: t[e0:e0 + el], ostd,
                                        gen, genf)
                else:
                    lw.w13 = self._param((a.num_experts, 2 * self.inter, h), (a.num_experts, 2 * big, h),
                                         self.shard_gate_up, std, gen, genf)
                    lw.w2 = self._param((a.num_experts, h, self.inter), (a.num_experts, h, big),
                                        lambda t: self.shard_cols(t, self.inter), ostd, gen, genf)
            else:
                lw.gate_up = self._param((2 * self.inter, h), (2 * big, h), self.shard_gate_up, std, gen, genf)
                lw.down = self._param((h, self.inter), (h, big), lambda t: self.shard_cols(t, self.inter), ostd,
                                      gen, genf)
            self.layers.append(lw)
        self.norm = torch.ones(h, dtype=self.dtype, device=self.device)
        self.lm_head = self._param((self.vocab_local, h), (a.vocab_size, h),
                                   lambda t: self.shard_rows(t, self.vocab_local), std, gen, genf)
        self.norms_folded = False
        self.fold_norm_weights()

    def fold_norm_weights(self, layers: Optional[List[int]] = None) -> None:
        """Fold each dense layer's RMSNorm weights into the projection that consumes the
        normalised activations: Wqkv <- Wqkv * ln1 (per input feature), Wgate_up <- Wgate_up *
        ln2, and the norm weights become ones. Mathematically a no-op (rmsnorm(x) * g @ W^T ==
        rmsnorm(x) @ (W * g)^T); it lets the decode fast path apply the norm as a per-row
        scale inside the GEMM / attention kernels (no norm kernels in the decode layer).
        Mixtral folds only ln1 (its ln2 output also feeds the router, so the MoE block keeps an
        explicit RMSNorm)."""
        for i, lw in enumerate(self.layers):
            if layers is not None and i not in layers:
                continue
            if not bool((lw.ln1 == 1).all()):
                lw.qkv.mul_(lw.ln1.to(lw.qkv.dtype)[None, :])
                lw.ln1.fill_(1)
            if self.arch.is_moe:
                continue
            if not bool((lw.ln2 == 1).all()):
                lw.gate_up.mul_(lw.ln2.to(lw.gate_up.dtype)[None, :])
                lw.ln2.fill_(1)
        self.norms_folded = True

    # LM head tiles tried in order (bench/micro_tp_tiles.py --shapes lm_head, cold, 32 rows: tile-order
    # (128, 128) 171.8 us vs the row-major (64, 256) 187.0 us for Llama-3's 128,256 x 4,096)
    LM_HEAD_TILES = ((128, 128), (64, 256), (64, 128))

    def pack_lm_head(self) -> bool:
        """Re-lay the LM head IN PLACE in the decode GEMM's tile order (one copy: its only consumer is the
        decode GEMM — logits are computed for the sampled rows, in <= 128-row chunks). Returns whether packed."""
        if self.lm_head_tile is not None:
            return True
        # packed in place (no second copy), so even a model that keeps its layers row-major for KV capacity
        # (EngineConfig.decode_weight_layout = single) gets the tile-order head and its greedy candidates
        if not (self.device.type == "cuda" and ops.native_available()):
            return False
        rows, k = self.lm_head.shape
        for wr, kc in self.LM_HEAD_TILES:
            if rows % wr == 0 and k % kc == 0 and ops.gd_tile_valid(wr, kc, 32):
                self.lm_head.copy_(ops.gd_pack_weights(self.lm_head, wr, kc=kc))
                self.lm_head_tile = (wr, kc)
                torch.cuda.empty_cache()  # the packing transients, before the KV pool is sized
                return True
        return False

    def lm_head_rows(self) -> torch.Tensor:
        """The LM head in its row-major layout (a copy when it is kept in tile order)."""
        if self.lm_head_tile is None:
            return self.lm_head
        return ops.gd_unpack_weights(self.lm_head, *self.lm_head_tile)

    def load_state_dict(self, tensors: Dict[str, torch.Tensor], fold: bool = True) -> int:
        """Load HuggingFace-named Llama / Mixtral tensors at their FULL (unsharded) shapes; this
        rank's Megatron slice is cut here, so a checkpoint shard file can be streamed in as is and
        q / k / v (gate / up, w1 / w3) may arrive in different calls. Returns the number of
        tensors consumed. ``fold``: fold the norm weights into Wqkv / Wgate_up afterwards (pass
        False while streaming several files, then call :meth:`fold_norm_weights` once)."""
        for lw in self.layers:  # decode tile-order copies go stale: re-packed by alloc_decode_scratch
            lw.tiled = {}
        if self.lm_head_tile is not None:  # back to row-major for the checkpoint's rows (re-packed likewise)
            self.lm_head.copy_(self.lm_head_rows())
            self.lm_head_tile = None
        a, d, r, ws = self.arch, self.head_dim, self.tp.rank, self.tp.world_size
        hq, hkv, inter = self.hq, self.hkv, self.inter
        kv_idx = (r * hkv) if a.num_kv_heads >= ws else r // (ws // a.num_kv_heads)
        n = 0

        def put(dst: torch.Tensor, src: torch.Tensor) -> None:
            nonlocal n
            dst.copy_(src.to(dst.device, dst.dtype))
            n += 1

        def rows(t, lo, cnt):
            return t[lo:lo + cnt]

        for name, t in tensors.items():
            if name == "model.embed_tokens.weight":
                put(self.embed, t)
                if a.tie_embeddings and "lm_head.weight" not in tensors:
                    put(self.lm_head, rows(t, r * self.vocab_local, self.vocab_local) if self.vocab_parallel else t)
                    n -= 1
            elif name == "model.norm.weight":
                put(self.norm, t)
            elif name == "lm_head.weight":
                put(self.lm_head, rows(t, r * self.vocab_local, self.vocab_local) if self.vocab_parallel else t)
            elif name.startswith("model.layers."):
                parts = name.split(".")
                li, rest = int(parts[2]), ".".join(parts[3:])
                if li >= len(self.layers):
                    continue
                lw = self.layers[li]
                if rest == "self_attn.q_proj.weight":
                    put(lw.qkv[: hq * d], rows(t, r * hq * d, hq * d))
                elif rest == "self_attn.k_proj.weight":
                    put(lw.qkv[hq * d:(hq + hkv) * d], rows(t, kv_idx * d, hkv * d))
                elif rest == "self_attn.v_proj.weight":
                    put(lw.qkv[(hq + hkv) * d:], rows(t, kv_idx * d, hkv * d))
                elif rest == "self_attn.o_proj.weight":
                    put(lw.o, t[:, r * hq * d:(r + 1) * hq * d])
                elif rest == "input_layernorm.weight":
                    put(lw.ln1, t)
                elif rest == "post_attention_layernorm.weight":
                    put(lw.ln2, t)
                elif rest == "mlp.gate_proj.weight" and not a.is_moe:
                    put(lw.gate_up[:inter], rows(t, r * inter, inter))
                elif rest == "mlp.up_proj.weight" and not a.is_moe:
                    put(lw.gate_up[inter:], rows(t, r * inter, inter))
                elif rest == "mlp.down_proj.weight" and not a.is_moe:
                    put(lw.down, t[:, r * inter:(r + 1) * inter])
                elif rest == "block_sparse_moe.gate.weight" and a.is_moe:
                    put(lw.router, t)
                elif rest.startswith("block_sparse_moe.experts.") and a.is_moe:
                    x, wname = int(parts[5]), parts[6]
                    if self.ep:  # whole experts: keep ours, rebased
                        if not self.expert0 <= x < self.expert0 + self.experts_local:
                            continue
                        x -= self.expert0
                        if wname == "w1":
                            put(lw.w13[x, :inter], t)
                        elif wname == "w3":
                            put(lw.w13[x, inter:], t)
                        elif wname == "w2":
                            put(lw.w2[x], t)
                    elif wname == "w1":
                        put(lw.w13[x, :inter], rows(t, r * inter, inter))
                    elif wname == "w3":
                        put(lw.w13[x, inter:], rows(t, r * inter, inter))
                    elif wname == "w2":
                        put(lw.w2[x], t[:, r * inter:(r + 1) * inter])
        if fold:
            self.fold_norm_weights()  # checkpoint norm weights -> folded into Wqkv / Wgate_up
        return n

    def reference_copy(self, device="cpu", dtype=torch.float32) -> "CausalLM":
        """This model's weights (same shard, same folded norms) converted to ``dtype`` on ``device``.
        On the CPU it runs on the plain-PyTorch reference ops (:mod:`src.ops.reference`): the fp32
        oracle the GPU engine is checked against at the served shapes (tests/test_oracle_gpu.py).
        The decode-GEMM tile-order copies are not carried over (they are a GPU layout)."""
        m = object.__new__(CausalLM)
        m.__dict__.update({k: v for k, v in self.__dict__.items()
                           if k not in ("layers", "embed", "norm", "lm_head", "cos_sin")})
        m.device, m.dtype = torch.device(device), dtype

        def conv(t):
            return None if t is None else t.detach().to(device=device, dtype=dtype)

        m.embed, m.norm, m.lm_head = conv(self.embed), conv(self.norm), conv(self.lm_head_rows())
        m.lm_head_tile = None
        m.layers = []
        for lw in self.layers:
            nl = LayerWeights()
            for s in ("ln1", "ln2", "qkv", "o", "gate_up", "down", "router", "w13", "w2"):
                setattr(nl, s, conv(getattr(lw, s)))
            m.layers.append(nl)
        m.cos_sin = self.cos_sin.to(device)
        return m

    def weight_bytes(self) -> int:
        tot = self.embed.numel() + self.lm_head.numel() + self.norm.numel()
        for lw in self.layers:
            for s in LayerWeights.__slots__:
                t = getattr(lw, s)
                if isinstance(t, torch.Tensor):
                    tot += t.numel()
        return tot * self.embed.element_size()

    # --------------------------------------------------------------- forward
    def forward(self, input_ids: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata,
                kv_pool: torch.Tensor) -> torch.Tensor:
        """Returns the final-norm hidden states [T, H]. ``kv_pool`` is
        [layers, 2, num_blocks, hkv, block_size, head_dim]."""
        eps = self.arch.rms_eps
        if (self._slab_path(input_ids) and meta.scratch is not None and not meta.is_prefill
                and self._fused_decode_ok(kv_pool, input_ids.shape[0])):
            if meta.pre_embedded and "h_in" in meta.scratch:
                residual, ssp0 = meta.scratch["h_in"][: input_ids.shape[0]], meta.scratch["ssp0"]
            else:  # the embedding gather and the first norm's row statistics in one launch
                residual, ssp0 = ops.embed_sumsq(input_ids, self.embed, meta.scratch["ssp0"])
            return self._forward_decode_fused(residual, positions, meta, kv_pool, ssp0=ssp0)
        residual = F.embedding(input_ids, self.embed)
        if self._slab_path(input_ids):
            if not self.tp.enabled and not self.arch.is_moe:  # the slab fallback is dense-only
                return self._forward_decode_slab(residual, positions, meta, kv_pool)
        if self.sequence_parallel and meta.is_prefill:
            return self._forward_sp(residual, positions, meta, kv_pool)
        if self._prefill_row_scale(residual, meta):
            return self._forward_prefill_row_scale(residual, positions, meta, kv_pool)
        x = ops.rms_norm(residual, self.layers[0].ln1, eps)
        h = None
        last = len(self.layers) - 1
        for li, lw in enumerate(self.layers):
            if li > 0:
                x = ops.fused_add_rms_norm(h, residual, lw.ln1, eps)
            if li == last and meta.is_prefill and meta.keep_rows is not None:
                return self._last_layer_kept_rows(lw, x, residual, positions, meta, kv_pool)
            attn = self._attention(li, lw, x, positions, meta, kv_pool)
            if meta.kv_hook is not None:  # layer li's KV is written: e.g. queue its overlapped export
                meta.kv_hook(li)
            o = self.tp.all_reduce(ops.linear(attn, lw.o))
            x = ops.fused_add_rms_norm(o, residual, lw.ln2, eps)
            h = self.tp.all_reduce(self._mlp(lw, x))
        return ops.fused_add_rms_norm(h, residual, self.norm, eps)

    def _prefill_row_scale(self, residual: torch.Tensor, meta: AttnMetadata) -> bool:
        """GPU prefill steps above decode sizes with the norm weights folded run the RMSNorms as row scales."""
        return (meta.is_prefill and residual.is_cuda and self.norms_folded and self.head_dim == 128
                and residual.shape[0] > ops.DECODE_GEMM_MAX_M)

    def _forward_prefill_row_scale(self, residual: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata,
                                   kv_pool: torch.Tensor) -> torch.Tensor:
        """Prefill with every folded RMSNorm as a per-token row scale: one pass adds the block output into the
        residual and writes rs = rsqrt(mean(residual^2) + eps) (``ops.rms_row_scale``); the qkv and gate/up
        projections run on the raw residual (their norm weights are folded in) and the consumers of their
        outputs apply rs — k / v in the RoPE + KV-write kernel, q in the attention's Q load, gate / up in SiLU *
        up. No normalised copy of the residual is written or read back: two [T, hidden] bf16 passes less per
        norm. Mixtral keeps its explicit ln2 (it also feeds the router)."""
        a, eps = self.arch, self.arch.rms_eps
        # one GPU (no all-reduce between a projection and its residual add): o and down add into the residual in
        # the GEMM epilogue, and the norm pass only reads the residual for its statistics
        gemm_resid = self.prefill_gemm_residual and not self.tp.enabled and not a.is_moe
        rs = ops.rms_row_scale(residual, None, eps)
        h = None
        last = len(self.layers) - 1
        for li, lw in enumerate(self.layers):
            if li > 0:
                rs = ops.rms_row_scale(residual, h, eps, out=rs)
            if li == last and meta.keep_rows is not None:
                return self._last_layer_kept_rows(lw, residual, residual, positions, meta, kv_pool, rs=rs)
            attn = self._attention(li, lw, residual, positions, meta, kv_pool, rs=rs)
            if meta.kv_hook is not None:
                meta.kv_hook(li)
            if gemm_resid:
                ops.linear_residual(residual, attn, lw.o)
                rs2 = ops.rms_row_scale(residual, None, eps)
                act = ops.silu_and_mul(ops.linear(residual, lw.gate_up), row_scale=rs2)
                ops.linear_residual(residual, act, lw.down)
                continue
            o = self.tp.all_reduce(ops.linear(attn, lw.o))
            if a.is_moe:
                x = ops.fused_add_rms_norm(o, residual, lw.ln2, eps)
                h = self.tp.all_reduce(self._mlp(lw, x))
            else:
                rs2 = ops.rms_row_scale(residual, o, eps)
                act = ops.silu_and_mul(ops.linear(residual, lw.gate_up), row_scale=rs2)
                h = self.tp.all_reduce(ops.linear(act, lw.down))
        if h is None:
            return ops.rms_norm(residual, self.norm, eps)
        return ops.fused_add_rms_norm(h, residual, self.norm, eps)

    def _last_layer_kept_rows(self, lw: LayerWeights, x: torch.Tensor, residual: torch.Tensor,
                              positions: torch.Tensor, meta: AttnMetadata, kv_pool: torch.Tensor,
                              rs: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Prefill's last layer, pruned to the rows whose hidden state is sampled: K / V of every token are
        still projected and written to the cache (later steps attend to them), but the query, attention, o, MLP
        and final norm run for one row per sampled sequence — the other rows' last-layer outputs would be
        discarded (a 16,384-token prefill of 32 prompts keeps 32 rows: ~1/32 of a layer's GEMM work for the
        sampled rows instead of a whole layer). The kept rows are each sequence's last token, so the attention is
        a 1-query-per-sequence prefill attention over the full context. rs: x is the raw residual and rs its
        RMSNorm row scales (:meth:`_forward_prefill_row_scale`)."""
        eps, d, hq, hkv = self.arch.rms_eps, self.head_dim, self.hq, self.hkv
        li = len(self.layers) - 1
        keep = meta.keep_rows
        n = keep.numel()
        qkv = ops.linear(x, lw.qkv)
        k_cache, v_cache = kv_pool[li, 0], kv_pool[li, 1]
        fuse_q = qkv.is_cuda
        ops.rope_and_cache(qkv, positions, self.cos_sin, meta.slot_mapping, k_cache, v_cache, hq, hkv, d,
                           rot_q=not fuse_q, row_scale=rs)
        if meta.kv_hook is not None:
            meta.kv_hook(li)
        if n == 0:
            return residual[:0]
        # the sequence of each kept row (rows of sequence i: [cu_q[i], cu_q[i + 1]))
        seq = torch.searchsorted(meta.cu_q[1:].to(torch.int64), keep, right=True)
        q = qkv.index_select(0, keep)[:, : hq * d].contiguous()
        cu1 = torch.arange(n + 1, dtype=torch.int32, device=q.device)
        attn = ops.attn_prefill(q, k_cache, v_cache, meta.block_tables.index_select(0, seq),
                                cu1, meta.ctx_lens.index_select(0, seq), 1, hq, hkv, self.scale,
                                cos_sin=self.cos_sin if fuse_q else None,
                                q_scale=rs.index_select(0, keep) if rs is not None else None)
        res = residual.index_select(0, keep)
        o = self.tp.all_reduce(ops.linear(attn, lw.o))
        x2 = ops.fused_add_rms_norm(o, res, lw.ln2, eps)
        h = self.tp.all_reduce(self._mlp(lw, x2))
        return ops.fused_add_rms_norm(h, res, self.norm, eps)

    def _attention(self, li: int, lw: LayerWeights, x: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata,
                   kv_pool: torch.Tensor, rs: Optional[torch.Tensor] = None) -> torch.Tensor:
        """qkv projection, RoPE + paged KV write, paged attention (prefill or decode) -> [T, hq*d].
        rs (GPU prefill): x is the raw residual and rs its per-token RMSNorm scale, applied to k / v in the
        KV write and to q in the attention's Q load."""
        d, hq, hkv = self.head_dim, self.hq, self.hkv
        qkv = ops.linear(x, lw.qkv)
        k_cache, v_cache = kv_pool[li, 0], kv_pool[li, 1]
        # prefill on the GPU: q's RoPE happens in the attention kernel's Q load (no q round trip through HBM)
        fuse_q = meta.is_prefill and qkv.is_cuda
        ops.rope_and_cache(qkv, positions, self.cos_sin, meta.slot_mapping, k_cache, v_cache, hq, hkv, d,
                           rot_q=not fuse_q, row_scale=rs)
        q = qkv[:, : hq * d]
        if meta.is_prefill:
            return ops.attn_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.ctx_lens,
                                    meta.max_q_len, hq, hkv, self.scale, cos_sin=self.cos_sin if fuse_q else None,
                                    q_scale=rs)
        return ops.attn_decode(q, k_cache, v_cache, meta.block_tables, meta.ctx_lens, meta.max_ctx, hq, hkv,
                               self.scale, part_o=meta.part_o, part_ml=meta.part_ml, counters=meta.attn_cnt)

    def _mlp(self, lw: LayerWeights, x: torch.Tensor) -> torch.Tensor:
        """This rank's partial FFN / MoE output (summed over the TP group by the caller)."""
        a = self.arch
        if a.is_moe:
            w, ids = ops.moe_route(x, lw.router, a.top_k)  # one fused launch at decode sizes
            return ops.moe_forward_routed(x, lw.w13, lw.w2, w, ids, expert0=self.expert0 if self.ep else None)
        return ops.linear(ops.linear_silu_mul(x, lw.gate_up), lw.down)

    def _forward_sp(self, residual_full: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata,
                    kv_pool: torch.Tensor) -> torch.Tensor:
        """Sequence-parallel prefill: this rank keeps tokens [r*n, (r+1)*n) of the residual stream
        (rows padded to a multiple of the TP size); projections and attention see all tokens."""
        tp, eps = self.tp, self.arch.rms_eps
        T = residual_full.shape[0]
        W = tp.world_size
        n = -(-T // W)
        pad = n * W - T

        def padded(t: torch.Tensor) -> torch.Tensor:
            return F.pad(t, (0, 0, 0, pad)) if pad else t

        residual = padded(residual_full)[tp.rank * n:(tp.rank + 1) * n].contiguous()
        x_s = ops.rms_norm(residual, self.layers[0].ln1, eps)
        h_s = None
        for li, lw in enumerate(self.layers):
            if li > 0:
                x_s = ops.fused_add_rms_norm(h_s, residual, lw.ln1, eps)
            attn = self._attention(li, lw, tp.all_gather_rows(x_s)[:T], positions, meta, kv_pool)
            o_s = tp.reduce_scatter_rows(padded(ops.linear(attn, lw.o)))
            x_s = ops.fused_add_rms_norm(o_s, residual, lw.ln2, eps)
            h_s = tp.reduce_scatter_rows(padded(self._mlp(lw, tp.all_gather_rows(x_s)[:T])))
        return tp.all_gather_rows(ops.fused_add_rms_norm(h_s, residual, self.norm, eps))[:T]

    # ------------------------------------------------- decode fast path (M <= 128)
    def _slab_path(self, input_ids: torch.Tensor) -> bool:
        """Decode-sized steps on the GPU run every projection on the weight-streaming kernel
        (split-K fp32 slabs reduced inside the consumer kernels; no separate reduction or SiLU
        launches). The slab fallback is TP=1 only; the fused path also serves TP."""
        if not (input_ids.is_cuda and ops.native_available()):
            return False
        m, h = input_ids.shape[0], self.arch.hidden_size
        return (1 <= m <= ops.DECODE_GEMM_MAX_M and h % 256 == 0 and self.inter % 256 == 0
                and (self.hq * self.head_dim) % 256 == 0 and self.layers[0].qkv.shape[0] % 32 == 0)

    def _forward_decode_slab(self, residual, positions, meta: AttnMetadata, kv_pool):
        a, eps, d = self.arch, self.arch.rms_eps, self.head_dim
        hq, hkv = self.hq, self.hkv
        x = ops.rms_norm(residual, self.layers[0].ln1, eps)
        slab = None
        for li, lw in enumerate(self.layers):
            if li > 0:
                x = ops.fused_add_rms_norm_slab(slab, residual, lw.ln1, eps)
            k_cache, v_cache = kv_pool[li, 0], kv_pool[li, 1]
            q = ops.rope_and_cache_slab(ops.linear_slab(x, lw.qkv), positions, self.cos_sin, meta.slot_mapping,
                                        k_cache, v_cache, hq, hkv, d)
            if meta.is_prefill:
                attn = ops.attn_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.ctx_lens,
                                        meta.max_q_len, hq, hkv, self.scale)
            else:
                attn = ops.attn_decode(q, k_cache, v_cache, meta.block_tables, meta.ctx_lens, meta.max_ctx, hq,
                                       hkv, self.scale, part_o=meta.part_o, part_ml=meta.part_ml,
                                       counters=meta.attn_cnt)
            x = ops.fused_add_rms_norm_slab(ops.linear_slab(attn, lw.o), residual, lw.ln2, eps)
            slab = ops.linear_slab(ops.linear_silu_mul(x, lw.gate_up), lw.down)
        return ops.fused_add_rms_norm_slab(slab, residual, self.norm, eps)

    # ----------------------------------------- fused decode path (norms folded, M <= 128)
    @staticmethod
    def decode_bucket(m: int) -> int:
        """Row bucket of a decode step: the activation image of its GEMMs (32, 64 or 128 rows)."""
        return 32 if m <= 32 else (64 if m <= 64 else 128)

    def decode_plan(self, m: int = 32) -> dict:
        """Decode-GEMM tiles of the fused path for steps of ``m`` rows: (wr, kc, sk) of the qkv slab
        projection and of the residual-updating o / down projections (wr in {32, 64, 128}: one
        norm-statistics tile per wr output columns), (wr, kc) of the gate/up projection."""
        h, d = self.arch.hidden_size, self.head_dim
        b = self.decode_bucket(m)
        # the fused attention stages sk x (G + 2) slab rows of 512 B (+ 2 KiB) in its 27 KiB merge
        # area (V3_MERGE_BYTES): at most 50 rows
        g = max(1, self.hq // self.hkv)
        rm = not getattr(self, "tiled_decode_weights", True)  # decode streams the row-major weights by choice (KV capacity)
        qkv = ops.decode_tile(self.layers[0].qkv.shape[0], h, 2, b, max_sk=max(1, 50 // (g + 2)), row_major=rm)
        # residual-updating split-K (mode 3); under TP the same tiles carry the one-shot exchange of each column
        # tile in their last arrivers' epilogue (one launch per row-parallel projection) where the group allows
        # it (TPContext.fused_row_parallel), else bf16 partial sums (mode 0) for a separate all-reduce launch
        o = ops.decode_tile(h, self.hq * d, 3, b, row_major=rm)
        down = ops.decode_tile(h, self.inter, 3, b, row_major=rm) if not self.arch.is_moe else None
        tp_fused = o_half = down_half = False
        if self.tp.enabled:
            fo = self._tp_fused_tile(h, self.hq * d, b, o) if not self.arch.is_moe else None
            fd = self._tp_fused_tile(h, self.inter, b, down) if fo is not None else None
            tp_fused = fo is not None and fd is not None
            if tp_fused:
                (o, o_half), (down, down_half) = fo, fd
            else:
                o = ops.decode_tile(h, self.hq * d, 0, b)
                down = ops.decode_tile(h, self.inter, 0, b) if not self.arch.is_moe else None
        gu = ops.decode_tile_silu(self.inter, h, b, row_major=rm) if not self.arch.is_moe else None
        return {"qkv": qkv, "o": o, "down": down, "gate_up": gu[:2] if gu else None,
                "gate_up_sk": gu[2] if gu else 1, "tp_fused": tp_fused, "o_half": o_half, "down_half": down_half}

    @torch.inference_mode()
    def calibrate_tp_exchange(self, iters: int = 20, force: bool = False) -> Optional[dict]:
        """Measure, on this TP group's links, the decode layer's two row-parallel projections (o, down; 32 rows) as
        ONE launch whose tiles carry the exchange against the separate form (bf16 partial GEMM + the one-shot
        all-reduce / residual / statistics launch), and keep the faster for serving (``tp.fused_preferred``; every
        rank takes the slowest rank's times, so the group agrees). Runs at engine build on a node (one rank per
        GPU); ranks sharing one GPU contend for the same CUs, so their timing says nothing about a node (``force``:
        tests). Every rank must call it. Returns the timings, or None when not measured."""
        import torch.distributed as dist

        tp = self.tp
        car = getattr(tp, "car", None)
        if not (tp.enabled and car is not None and self.device.type == "cuda" and not self.arch.is_moe):
            return None
        if car.ranks_per_gpu > 1 and not force:
            return None
        tp.fused_preferred = None
        plan = self.decode_plan(32)
        if not plan["tp_fused"]:
            return None  # the residency rule already keeps the separate launch
        h, dev = self.arch.hidden_size, self.device
        g = torch.Generator(device=dev).manual_seed(11 + tp.rank)
        res = {}
        fused_t = sep_t = 0.0
        for name, k, half in (("o", self.hq * self.head_dim, plan["o_half"]), ("down", self.inter, plan["down_half"])):
            wr, kc, sk = plan[name]
            x = (torch.randn(32, k, device=dev, generator=g) * 0.5).to(self.dtype)
            w = (torch.randn(h, k, device=dev, generator=g) * 0.02).to(self.dtype)
            resid = torch.zeros(32, h, dtype=self.dtype, device=dev)
            ssp = torch.zeros(h // wr, ops.SSP_LD, dtype=torch.float32, device=dev)
            ssp1 = torch.zeros(1, ops.SSP_LD, dtype=torch.float32, device=dev)
            cnt = torch.zeros(h // wr, dtype=torch.int32, device=dev)

            # both forms on tile-order weights, as served (the separate form's partial GEMM on its own mode-0 tile)
            wt = ops.gd_pack_weights(w, wr, kc=kc)
            wr0, kc0 = ops.decode_tile(h, k, 0, 32)[:2]
            wt0 = ops.gd_pack_weights(w, wr0, kc=kc0)

            def fused():
                tp.row_parallel_residual(x, wt, resid, ssp, cnt, wr, kc, sk, tiled=True, half_ring=half)

            def separate():
                tp.all_reduce_residual(ops.linear_tiled(x, wt0, wr0, kc0), resid, ssp1)

            times = []
            for fn in (fused, separate):
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize(dev)
                e0.record()
                for _ in range(iters):
                    fn()
                e1.record()
                torch.cuda.synchronize(dev)
                times.append(e0.elapsed_time(e1) * 1e3 / iters)
            res[name] = {"fused_us": round(times[0], 2), "separate_us": round(times[1], 2)}
            fused_t += times[0]
            sep_t += times[1]
        t = torch.tensor([fused_t, sep_t], dtype=torch.float64)
        grp = tp.cpu_group if tp.cpu_group is not None else tp.group
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=grp)  # the group's slowest rank decides, identically on all
        tp.fused_preferred = bool(t[0] <= t[1])
        res.update(fused_total_us=round(float(t[0]), 2), separate_total_us=round(float(t[1]), 2),
                   fused_preferred=tp.fused_preferred)
        if car.error():
            raise RuntimeError("TP exchange calibration: a one-shot collective timed out")
        return res

    def _tp_fused_tile(self, n: int, k: int, bucket: int, tile):
        """((wr, kc, sk), half_ring) of a row-parallel projection whose tiles carry the TP exchange, or None. The
        measured tile first (with its full LDS ring, then — at <= 32 rows — the half-LDS ring that puts two
        workgroups on a CU), then wider tiles (fewer waiting last arrivers): the first that passes the group's
        residency rule (custom_allreduce.fused_exchange_ok, on the instantiation's real occupancy)."""
        lim = ops.SSP_MAX_TILES if bucket <= 32 else ops.SSP_MAX_TILES_WIDE
        cands = [tuple(tile)] + [c for c in ((64, 256, 1), (64, 128, 1), (64, 128, 2), (128, 128, 1), (128, 128, 2))
                                 if c != tuple(tile)]
        for wr, kc, sk in cands:
            if n % wr or k % (kc * sk) or n // wr > lim or not ops.gd_tile_valid(wr, kc, bucket):
                continue
            for half in ((False, True) if bucket <= 32 else (False,)):
                occ = ops.gd_occupancy(3, wr, kc, sk, bucket, half)
                if half and occ <= 0:
                    continue
                if self.tp.fused_row_parallel(n // wr, n // wr * sk, occ):
                    return (wr, kc, sk), half
        return None

    def _packed_layouts(self, buckets) -> set:
        """(projection, wr, kc) tile-order copies the fused path uses for these row buckets."""
        need = set()
        for b in buckets:
            p = self.decode_plan(b)
            need.add(("qkv", *p["qkv"][:2]))
            need.add(("gate_up", *p["gate_up"][:2]))
            need.add(("o", *p["o"][:2]))      # under TP: the row-parallel shards, plain bf16 tiles
            if p["down"] is not None:
                need.add(("down", *p["down"][:2]))
        return need

    def pack_decode_weights(self, buckets=(32,)) -> bool:
        """Keep copies of the dense projections in the decode GEMM's tile order (ops.gd_pack_weights:
        every LDS-DMA piece one linear 1-KiB read) for the fused decode path — one per (wr, kc) tile the
        row buckets' plans use; prefill keeps the row-major copies for hipBLASLt. Only done while the
        weights and their copies take <= 1/2 of the device memory (8B at batch <= 32: +13 GiB of 288 GB;
        at batch 128: +34 GiB). ``self.tiled_decode_weights = False`` keeps the decode GEMMs on the row-major
        weights (4 % slower bench, profiles/r5_decode_weight_layout_ab.txt)."""
        if not self.tiled_decode_weights or self.arch.is_moe or not self.norms_folded:
            return False
        if not (self.device.type == "cuda" and ops.native_available()):
            return False
        need, extra = self._decode_copy_plan(buckets)
        total = torch.cuda.get_device_properties(self.device).total_memory
        if self.weight_bytes() + extra > total // 2:
            return False
        for lw in self.layers:
            for name, wr, kc in need:
                if (name, wr, kc) not in lw.tiled:
                    lw.tiled[(name, wr, kc)] = ops.gd_pack_weights(getattr(lw, name), wr, silu=name == "gate_up",
                                                                   kc=kc)
        return True

    def _decode_copy_plan(self, buckets):
        """(tile layouts, bytes) of the tile-order decode weight copies these row buckets would use."""
        lw0 = self.layers[0]

        def tiles(name, wr, kc):  # the tile covers the (shard's) weight exactly
            rows, k = getattr(lw0, name).shape
            silu = name == "gate_up"
            return k % kc == 0 and (rows // 2 if silu else rows) % (wr // 2 if silu else wr) == 0

        need = {t for t in self._packed_layouts(buckets) if tiles(*t)}
        extra = sum(getattr(lw0, name).numel() * lw0.qkv.element_size() for name, _, _ in need) * len(self.layers)
        return need, extra

    def decode_copy_bytes(self, buckets) -> int:
        """HBM the tile-order decode weight copies would take (0 where none are made)."""
        if not self.tiled_decode_weights or self.arch.is_moe or not self.norms_folded:
            return 0
        return self._decode_copy_plan(buckets)[1]

    @staticmethod
    def decode_buckets(max_rows: int) -> List[int]:
        """Row buckets a decode batch of up to ``max_rows`` sequences can fall in."""
        top = CausalLM.decode_bucket(min(max(1, max_rows), ops.DECODE_GEMM_MAX_M))
        return [b for b in (32, 64, 128) if b <= top]

    def alloc_decode_scratch(self, max_rows: int = 32) -> Optional[dict]:
        if not (self.device.type == "cuda" and ops.native_available()):
            return None
        h = self.arch.hidden_size
        buckets = self.decode_buckets(max_rows)
        plans = {b: self.decode_plan(b) for b in buckets}
        f32, i32 = torch.float32, torch.int32
        # TP: the row-parallel projections are all-reduced first, then one kernel adds into the
        # residual and writes a single statistics tile (so does the MoE block's residual add)
        if self.tp.enabled and not any(p["tp_fused"] for p in plans.values()):
            to = td = 1
        else:
            to = max(h // p["o"][0] for p in plans.values())
            td = 1 if self.arch.is_moe else max(h // p["down"][0] for p in plans.values())
        # consumers take <= 256 statistics tiles at <= 32 rows, <= 128 above (gemm_decode.hip / attention.hip)
        for b, p in plans.items():
            lim = ops.SSP_MAX_TILES if b <= 32 else ops.SSP_MAX_TILES_WIDE
            if not (self.tp.enabled and not p["tp_fused"]) and max(h // p["o"][0],
                                                                   0 if self.arch.is_moe else h // p["down"][0]) > lim:
                return None
        dev = self.device
        self.pack_decode_weights(buckets)
        self.pack_lm_head()
        ld = ops.SSP_LD
        sc = {"plans": plans, "ssp0": torch.zeros(1, ld, dtype=f32, device=dev),
              # split-K gate/up (mode 6): fp32 partial slab + per-tile tickets, sized for the largest bucket
              "slab6": torch.empty(max((p["gate_up_sk"] * b * 2 * self.inter if p["gate_up_sk"] > 1 else 0)
                                       for b, p in plans.items()), dtype=f32, device=dev),
              "cnt6": torch.zeros(max((self.inter // (p["gate_up"][0] // 2) if p["gate_up"] else 0)
                                      for p in plans.values()), dtype=i32, device=dev),
              "ssp_a": torch.zeros(to, ld, dtype=f32, device=dev), "cnt_a": torch.zeros(to, dtype=i32, device=dev),
              "ssp_b": torch.zeros(td, ld, dtype=f32, device=dev), "cnt_b": torch.zeros(td, dtype=i32, device=dev),
              # the step's embedding rows when the previous step's sampling launch writes them (AttnMetadata.pre_embedded)
              "h_in": torch.zeros(max(buckets), h, dtype=self.dtype, device=dev)}
        return sc

    def _fused_decode_ok(self, kv_pool: torch.Tensor, m: int = 32) -> bool:
        g = self.hq // self.hkv
        sq = self.decode_plan(m)["qkv"][2]
        return (self.norms_folded and self.head_dim == 128 and kv_pool.shape[4] == 16 and g in (1, 2, 4, 8)
                and ((sq * (g + 2) + 1) // 2) * 1024 + 2048 <= V3_MERGE_BYTES)

    def _forward_decode_fused(self, h: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata,
                              kv_pool: torch.Tensor, ssp0: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Decode layer = 5 launches: qkv (split-K slabs) -> attention (norm scale + slab sum + RoPE
        + KV write in its prologue) -> o (slabs, last arriver adds into the residual and writes the
        next norm's row statistics) -> gate/up (norm as a row scale, SiLU*mul) -> down (as o).
        The residual stream `h` is updated in place; norm weights are folded into Wqkv / Wgate_up.
        Tiles come from the plan of the step's row bucket (32 / 64 / 128)."""
        a, eps = self.arch, self.arch.rms_eps
        sc = meta.scratch
        plan = sc["plans"][self.decode_bucket(h.shape[0])]
        hq, hkv, hid = self.hq, self.hkv, a.hidden_size
        (wq, kq, sq), (wo, ko, so) = plan["qkv"], plan["o"]
        # statistics tiles of the residual-updating projections (one per wr output columns; 1 under TP)
        tiles = not self.tp.enabled or plan["tp_fused"]  # per-tile statistics (mode 3), or one row-sum tile
        ssp_a = sc["ssp_a"][: hid // wo if tiles else 1]
        ssp_b = sc["ssp_b"]
        if tiles and not a.is_moe:
            ssp_b = ssp_b[: hid // plan["down"][0]]

        def tw(lw, name, wr, kc):  # (weight, tiled?) for this tile
            t = lw.tiled.get((name, wr, kc))
            return (getattr(lw, name), False) if t is None else (t, True)

        ssp_prev = ssp0 if ssp0 is not None else ops.row_sumsq(h, out=sc["ssp0"])
        for li, lw in enumerate(self.layers):
            k_cache, v_cache = kv_pool[li, 0], kv_pool[li, 1]
            wqkv, tq = tw(lw, "qkv", wq, kq)
            slab = ops.linear_slab(h, wqkv, sk=sq, wr=wq, tiled=tq, kc=kq)
            attn = ops.attn_decode_fused(slab, ssp_prev, positions, self.cos_sin, meta.slot_mapping,
                                         k_cache, v_cache, meta.block_tables, meta.ctx_lens, meta.max_ctx, hq, hkv,
                                         self.scale, eps, hid, meta.part_o, meta.part_ml, meta.attn_cnt)
            if a.is_moe:  # ln2 stays explicit (it also feeds the router); MoE output added back + statistics
                if self.tp.enabled:
                    self.tp.all_reduce_residual(ops.linear(attn, lw.o), h, ssp_a)
                else:
                    ops.linear_slab_residual(attn, lw.o, h, ssp_a, sc["cnt_a"], wo, so, kc=ko)
                x = ops.rms_norm(h, lw.ln2, eps)
                if self.tp.enabled:
                    self.tp.all_reduce_residual(self._mlp(lw, x), h, ssp_b)
                else:  # combine + residual add + statistics in one launch
                    wr_, ids_ = ops.moe_route(x, lw.router, a.top_k)
                    ops.moe_forward_routed(x, lw.w13, lw.w2, wr_, ids_, residual=h, ssp=ssp_b)
            else:
                wg, kg = plan["gate_up"]
                gsk = plan.get("gate_up_sk", 1)
                wgu, tg = tw(lw, "gate_up", wg, kg)
                if self.tp.enabled and plan["tp_fused"]:
                    # row-parallel GEMM + one-shot all-reduce + residual + statistics: one launch each
                    wdn_, kd, sd = plan["down"]
                    wo_t, to_ = tw(lw, "o", wo, ko)
                    wd_t, td_ = tw(lw, "down", wdn_, kd)
                    self.tp.row_parallel_residual(attn, wo_t, h, ssp_a, sc["cnt_a"], wo, ko, so, tiled=to_,
                                                  half_ring=plan["o_half"])
                    act = ops.linear_silu_mul_rownorm(h, wgu, ssp_a, eps, wg, tiled=tg, kc=kg, sk=gsk,
                                                      slab=sc["slab6"], counters=sc["cnt6"])
                    self.tp.row_parallel_residual(act, wd_t, h, ssp_b, sc["cnt_b"], wdn_, kd, sd, tiled=td_,
                                                  half_ring=plan["down_half"])
                elif self.tp.enabled:  # row-parallel partial sums -> all-reduce -> residual + statistics (one
                    # launch on the one-shot IPC path, see TPContext.all_reduce_residual)
                    self.tp.all_reduce_residual(self._row_parallel(attn, lw, "o", plan), h, ssp_a)
                    act = ops.linear_silu_mul_rownorm(h, wgu, ssp_a, eps, wg, tiled=tg, kc=kg, sk=gsk,
                                                      slab=sc["slab6"], counters=sc["cnt6"])
                    self.tp.all_reduce_residual(self._row_parallel(act, lw, "down", plan), h, ssp_b)
                else:
                    wdn_, kd, sd = plan["down"]
                    wo_t, to_ = tw(lw, "o", wo, ko)
                    wd_t, td_ = tw(lw, "down", wdn_, kd)
                    ops.linear_slab_residual(attn, wo_t, h, ssp_a, sc["cnt_a"], wo, so, tiled=to_, kc=ko)
                    act = ops.linear_silu_mul_rownorm(h, wgu, ssp_a, eps, wg, tiled=tg, kc=kg, sk=gsk,
                                                      slab=sc["slab6"], counters=sc["cnt6"])
                    ops.linear_slab_residual(act, wd_t, h, ssp_b, sc["cnt_b"], wdn_, sd, tiled=td_, kc=kd)
            ssp_prev = ssp_b
        return ops.rms_norm(h, self.norm, eps)

    @staticmethod
    def _row_parallel(x: torch.Tensor, lw, name: str, plan: dict) -> torch.Tensor:
        """TP decode: this rank's partial sum of a row-parallel projection, on its tile-order copy when
        one was packed for the step's row bucket (else the row-major weight)."""
        wr, kc = plan[name][:2]
        t = lw.tiled.get((name, wr, kc))
        return ops.linear(x, getattr(lw, name)) if t is None else ops.linear_tiled(x, t, wr, kc)

    def lm_head_argmax_parts(self) -> int:
        """Greedy candidates per row the LM head writes with its logits (one per column tile; 0: it cannot — the
        head is not in tile order, or is split over a TP group's vocabulary)."""
        if self.lm_head_tile is None or self.vocab_parallel:
            return 0
        return self.lm_head.shape[0] // self.lm_head_tile[0]

    def compute_logits(self, hidden: torch.Tensor, argmax_parts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """argmax_parts [>= rows, lm_head_argmax_parts(), 2] int32 (decode steps, <= 128 rows): also filled with the
        LM head's per-column-tile greedy candidates, which ops.sample(lm_part=...) reduces for greedy rows."""
        if argmax_parts is not None:  # the caller's argmax reads these candidates: never leave them stale
            if not (self.lm_head_argmax_parts() == argmax_parts.shape[1] and 0 < hidden.shape[0] <= ops.DECODE_GEMM_MAX_M):
                raise ValueError("LM-head argmax candidates requested where the head cannot write them")
            wr, kc = self.lm_head_tile
            return ops.linear_tiled_argmax(hidden, self.lm_head, wr, kc, argmax_parts[:hidden.shape[0]])
        if self.lm_head_tile is not None and hidden.shape[0] > 0:  # tile order: the decode GEMM, <= 128 rows
            wr, kc = self.lm_head_tile
            mx = ops.DECODE_GEMM_MAX_M
            logits = (ops.linear_tiled(hidden, self.lm_head, wr, kc) if hidden.shape[0] <= mx else
                      torch.cat([ops.linear_tiled(hidden[i:i + mx], self.lm_head, wr, kc)
                                 for i in range(0, hidden.shape[0], mx)]))
        else:
            logits = ops.linear(hidden, self.lm_head)
        if self.vocab_parallel:
            logits = self.tp.all_gather_last(logits)
        return logits
