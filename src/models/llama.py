"""
Llama-3 / Mixtral decoder on PyTorch-ROCm + the gfx950 kernels of :mod:`src.ops`.

Per decoder layer (T = tokens of the step):

    x   = fused_add_rms_norm(h, residual, ln1)          HIP  (residual += h in place)
    qkv = x @ Wqkv^T                                    hipBLASLt   [T, (hq+2hkv)*128]
    rope_and_cache(qkv → q rotated in place, k/v → paged HBM blocks)   HIP
    a   = attn_prefill | attn_decode (paged, GQA)       HIP  (MFMA)
    o   = a @ Wo^T   (+ all_reduce over RCCL if TP)     hipBLASLt
    x   = fused_add_rms_norm(o, residual, ln2)          HIP
    Llama:   d = silu_and_mul(x @ Wgu^T) @ Wd^T          hipBLASLt + HIP
    Mixtral: d = moe_forward(x, router)                  HIP routing + MFMA grouped GEMM
    (+ all_reduce if TP)

Weights are stored pre-fused ([q|k|v] and [gate|up]) so each projection is one
GEMM. Only the last token of each prefill sequence reaches the LM head.
The same module runs CPU tensors through :mod:`src.ops.reference` for tests.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

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


class LayerWeights:
    __slots__ = ("ln1", "ln2", "qkv", "o", "gate_up", "down", "router", "w13", "w2")

    def __init__(self):
        for s in self.__slots__:
            setattr(self, s, None)


class CausalLM:
    """A TP-sharded decoder-only LM (no nn.Module overhead on the hot path)."""

    def __init__(self, arch: ArchConfig, device, dtype=torch.bfloat16, tp: Optional[TPContext] = None,
                 seed: int = 0, init_std: float = 0.02, max_position: Optional[int] = None):
        self.arch = arch
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPContext()
        a, tpc = arch, self.tp
        self.hq = tpc.shard(a.num_heads)
        self.hkv = tpc.kv_heads(a.num_kv_heads)
        self.inter = tpc.shard(a.intermediate_size)
        self.vocab_local = tpc.shard(a.vocab_size) if a.vocab_size % tpc.world_size == 0 else a.vocab_size
        self.vocab_parallel = self.vocab_local != a.vocab_size
        self.head_dim = a.head_dim
        self.scale = 1.0 / math.sqrt(a.head_dim)
        self.max_position = max_position or a.max_position
        self.layers: List[LayerWeights] = []
        self._init_random(seed, init_std)
        self.cos_sin = rope_cos_sin(self.max_position, a.head_dim, a.rope_theta, self.device, a.rope_scaling)

    # ------------------------------------------------------------------ init
    def _randn(self, *shape, std: float, gen) -> torch.Tensor:
        t = torch.empty(*shape, dtype=self.dtype, device=self.device)
        t.normal_(0.0, std, generator=gen)
        return t

    def _init_random(self, seed: int, std: float) -> None:
        a = self.arch
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed * 7919 + self.tp.rank)
        h, d = a.hidden_size, a.head_dim
        # Embedding replicated on every rank: identical across ranks.
        gen_e = torch.Generator(device=self.device)
        gen_e.manual_seed(seed)
        self.embed = self._randn(a.vocab_size, h, std=1.0, gen=gen_e)
        for _ in range(a.num_layers):
            lw = LayerWeights()
            lw.ln1 = torch.ones(h, dtype=self.dtype, device=self.device)
            lw.ln2 = torch.ones(h, dtype=self.dtype, device=self.device)
            lw.qkv = self._randn((self.hq + 2 * self.hkv) * d, h, std=std, gen=gen)
            lw.o = self._randn(h, self.hq * d, std=std / math.sqrt(2 * a.num_layers), gen=gen)
            if a.is_moe:
                lw.router = self._randn(a.num_experts, h, std=std, gen=gen_e)  # replicated router
                lw.w13 = self._randn(a.num_experts, 2 * self.inter, h, std=std, gen=gen)
                lw.w2 = self._randn(a.num_experts, h, self.inter, std=std / math.sqrt(2 * a.num_layers), gen=gen)
            else:
                lw.gate_up = self._randn(2 * self.inter, h, std=std, gen=gen)
                lw.down = self._randn(h, self.inter, std=std / math.sqrt(2 * a.num_layers), gen=gen)
            self.layers.append(lw)
        self.norm = torch.ones(h, dtype=self.dtype, device=self.device)
        self.lm_head = self._randn(self.vocab_local, h, std=std, gen=gen)

    def load_state_dict(self, tensors: Dict[str, torch.Tensor]) -> int:
        """Load HF-named Llama/Mixtral weights (already TP-sliced by the caller
        when tp > 1). Returns the number of tensors consumed."""
        n = 0
        a = self.arch

        def take(name):
            nonlocal n
            t = tensors.get(name)
            if t is not None:
                n += 1
            return t

        e = take("model.embed_tokens.weight")
        if e is not None:
            self.embed.copy_(e)
        for i, lw in enumerate(self.layers):
            p = f"model.layers.{i}."
            q, k, v = take(p + "self_attn.q_proj.weight"), take(p + "self_attn.k_proj.weight"), take(p + "self_attn.v_proj.weight")
            if q is not None:
                lw.qkv.copy_(torch.cat([q, k, v], 0))
                lw.o.copy_(take(p + "self_attn.o_proj.weight"))
            for nm, dst in (("input_layernorm.weight", lw.ln1), ("post_attention_layernorm.weight", lw.ln2)):
                t = take(p + nm)
                if t is not None:
                    dst.copy_(t)
            if not a.is_moe:
                g, u = take(p + "mlp.gate_proj.weight"), take(p + "mlp.up_proj.weight")
                if g is not None:
                    lw.gate_up.copy_(torch.cat([g, u], 0))
                    lw.down.copy_(take(p + "mlp.down_proj.weight"))
            else:
                r = take(p + "block_sparse_moe.gate.weight")
                if r is not None:
                    lw.router.copy_(r)
                for x in range(a.num_experts):
                    q2 = p + f"block_sparse_moe.experts.{x}."
                    w1, w3, w2 = take(q2 + "w1.weight"), take(q2 + "w3.weight"), take(q2 + "w2.weight")
                    if w1 is not None:
                        lw.w13[x].copy_(torch.cat([w1, w3], 0))
                        lw.w2[x].copy_(w2)
        t = take("model.norm.weight")
        if t is not None:
            self.norm.copy_(t)
        t = take("lm_head.weight")
        if t is not None:
            self.lm_head.copy_(t)
        return n

    def weight_bytes(self) -> int:
        tot = self.embed.numel() + self.lm_head.numel() + self.norm.numel()
        for lw in self.layers:
            for s in LayerWeights.__slots__:
                t = getattr(lw, s)
                if t is not None:
                    tot += t.numel()
        return tot * self.embed.element_size()

    # --------------------------------------------------------------- forward
    def forward(self, input_ids: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata,
                kv_pool: torch.Tensor) -> torch.Tensor:
        """Returns the final-norm hidden states [T, H]. ``kv_pool`` is
        [layers, 2, num_blocks, hkv, block_size, head_dim]."""
        a = self.arch
        eps = a.rms_eps
        d = self.head_dim
        hq, hkv = self.hq, self.hkv
        residual = F.embedding(input_ids, self.embed)
        x = ops.rms_norm(residual, self.layers[0].ln1, eps)
        h = None
        for li, lw in enumerate(self.layers):
            if li > 0:
                x = ops.fused_add_rms_norm(h, residual, lw.ln1, eps)
            qkv = F.linear(x, lw.qkv)
            k_cache, v_cache = kv_pool[li, 0], kv_pool[li, 1]
            ops.rope_and_cache(qkv, positions, self.cos_sin, meta.slot_mapping, k_cache, v_cache, hq, hkv, d)
            q = qkv[:, : hq * d]
            if meta.is_prefill:
                attn = ops.attn_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.ctx_lens,
                                        meta.max_q_len, hq, hkv, self.scale)
            else:
                attn = ops.attn_decode(q, k_cache, v_cache, meta.block_tables, meta.ctx_lens, meta.max_ctx, hq,
                                       hkv, self.scale, part_o=meta.part_o, part_ml=meta.part_ml)
            o = self.tp.all_reduce(F.linear(attn, lw.o))
            x = ops.fused_add_rms_norm(o, residual, lw.ln2, eps)
            if a.is_moe:
                gating = F.linear(x, lw.router)
                h = ops.moe_forward(x, lw.w13, lw.w2, gating, a.top_k)
            else:
                h = F.linear(ops.silu_and_mul(F.linear(x, lw.gate_up)), lw.down)
            h = self.tp.all_reduce(h)
        return ops.fused_add_rms_norm(h, residual, self.norm, eps)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = F.linear(hidden, self.lm_head)
        if self.vocab_parallel:
            logits = self.tp.all_gather_last(logits)
        return logits
