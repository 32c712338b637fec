"""
Custom ops. GPU tensors always go to the hand-written gfx950 HIP kernels in
``src/_C*.so`` (built by :mod:`src._build`); if that extension is missing a
GPU call raises — there is no silent eager fallback on the GPU. CPU tensors use
:mod:`src.ops.reference` (the fp32 semantics the kernels are tested against),
which lets the engine's control flow run in CPU-only tests.
"""

from __future__ import annotations

from typing import Optional

import torch

from . import reference as ref

_C = None
_C_ERR: Optional[BaseException] = None
try:
    from src import _C  # type: ignore  # noqa: F811
except Exception as e:  # pragma: no cover - depends on build state
    _C_ERR = e


def native_available() -> bool:
    return _C is not None


def _kern():
    if _C is None:
        raise RuntimeError(
            "HIP kernel extension src/_C is not built or failed to load "
            f"({_C_ERR!r}); run `python -m src._build` (hipcc --offload-arch=gfx950)")
    return _C


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not x.is_cuda:
        r = ref.rms_norm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    _kern().rms_norm(out, x, w, eps)
    return out


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """residual += x (in place, bf16); returns rms_norm(residual) * w."""
    if not x.is_cuda:
        y, r = ref.fused_add_rms_norm(x, residual, w, eps)
        residual.copy_(r)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    _kern().fused_add_rms_norm(out, x, residual, w, eps)
    return out


def silu_and_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not x.is_cuda:
        return ref.silu_and_mul(x)
    if out is None:
        out = torch.empty(x.shape[0], x.shape[1] // 2, dtype=x.dtype, device=x.device)
    _kern().silu_and_mul(out, x)
    return out


def rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq: int, hkv: int, head_dim: int) -> None:
    if not qkv.is_cuda:
        ref.rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, head_dim)
        return
    _kern().rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, head_dim)


def attn_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_q_len: int, hq: int, hkv: int,
                 scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not q.is_cuda:
        return ref.attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, hq, hkv, scale).reshape(q.shape[0], -1)
    if out is None:
        out = torch.empty(q.shape[0], hq * 128, dtype=q.dtype, device=q.device)
    _kern().attn_prefill(out, q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_q_len, hq, hkv, scale)
    return out


def decode_partials(max_ctx: int) -> int:
    return int(_kern().decode_partials(max_ctx))


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, max_ctx: int, hq: int, hkv: int, scale: float,
                part_o: Optional[torch.Tensor] = None, part_ml: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not q.is_cuda:
        n = ctx_lens.numel()
        cu = torch.arange(n + 1, dtype=torch.int32)
        return ref.attention(q[:n], k_cache, v_cache, block_tables, cu, ctx_lens, hq, hkv, scale).reshape(n, -1)
    n = ctx_lens.numel()
    if out is None:
        out = torch.empty(n, hq * 128, dtype=q.dtype, device=q.device)
    if part_o is None or part_ml is None:
        maxp = decode_partials(max_ctx)
        part_o = torch.empty(n * hq * maxp * 128, dtype=torch.float32, device=q.device)
        part_ml = torch.empty(n * hq * maxp * 2, dtype=torch.float32, device=q.device)
    _kern().attn_decode(out, part_o, part_ml, q, k_cache, v_cache, block_tables, ctx_lens, max_ctx, hq, hkv, scale)
    return out


def sample(logits, temperature=None, top_k=None, top_p=None, seeds=None, steps=None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not logits.is_cuda:
        return ref.sample(logits, temperature, top_k, top_p, seeds, steps)
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    _kern().sample(out, logits, temperature, top_k, top_p, seeds, steps)
    return out


def copy_blocks(pool: torch.Tensor, pairs: torch.Tensor) -> None:
    """pool viewed [planes, num_blocks, ...]; pairs [n, 2] int64 (src, dst)."""
    if not pool.is_cuda:
        for s, d in pairs.tolist():
            pool[:, d] = pool[:, s]
        return
    _kern().copy_blocks(pool, pairs)


def gather_blocks(pool: torch.Tensor, ids: torch.Tensor, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Pack blocks `ids` of every plane into [n, planes, slab] (KV transfer staging)."""
    planes, nb = pool.shape[0], pool.shape[1]
    slab = pool.numel() // (planes * nb)
    if buf is None:
        buf = torch.empty(ids.numel(), planes, slab, dtype=pool.dtype, device=pool.device)
    if not pool.is_cuda:
        buf.copy_(pool.reshape(planes, nb, slab)[:, ids.long()].transpose(0, 1))
        return buf
    _kern().move_blocks(pool, buf, ids, True)
    return buf


def scatter_blocks(pool: torch.Tensor, ids: torch.Tensor, buf: torch.Tensor) -> None:
    planes, nb = pool.shape[0], pool.shape[1]
    slab = pool.numel() // (planes * nb)
    if not pool.is_cuda:
        pool.view(planes, nb, slab)[:, ids.long()] = buf.view(ids.numel(), planes, slab).transpose(0, 1)
        return
    _kern().move_blocks(pool, buf, ids, False)


def topk_softmax(gating: torch.Tensor, k: int, renorm: bool = True):
    if not gating.is_cuda:
        return ref.topk_softmax(gating, k, renorm)
    t = gating.shape[0]
    w = torch.empty(t, k, dtype=torch.float32, device=gating.device)
    ids = torch.empty(t, k, dtype=torch.int32, device=gating.device)
    _kern().topk_softmax(w, ids, gating, renorm)
    return w, ids


def moe_align(ids: torch.Tensor, num_experts: int):
    """Expert-sorted order of the flattened (token, slot) assignments."""
    n = ids.numel()
    dev = ids.device
    offsets = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
    sorted_idx = torch.empty(n, dtype=torch.int32, device=dev)
    pos = torch.empty(n, dtype=torch.int32, device=dev)
    _kern().moe_align(offsets, sorted_idx, pos, ids.reshape(-1).contiguous(), num_experts)
    return offsets, sorted_idx, pos


def moe_forward(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, gating: torch.Tensor, k: int,
                renorm: bool = True) -> torch.Tensor:
    """Fused-routing MoE FFN on the HIP kernels: route → align → gather →
    grouped GEMM (gate/up) → SiLU·mul → grouped GEMM (down) → weighted combine.
    No host synchronisation (hipGraph-capturable)."""
    if not x.is_cuda:
        return ref.moe_forward(x, w13, w2, gating, k, renorm)
    kern = _kern()
    t, hdim = x.shape
    e = w13.shape[0]
    w, ids = topk_softmax(gating, k, renorm)
    offsets, sorted_idx, pos = moe_align(ids, e)
    xs = torch.empty(t * k, hdim, dtype=x.dtype, device=x.device)
    kern.moe_gather(xs, x, sorted_idx, k)
    h = torch.empty(t * k, w13.shape[1], dtype=x.dtype, device=x.device)
    kern.moe_grouped_gemm(h, xs, w13, offsets)
    a = silu_and_mul(h)
    ys = torch.empty(t * k, hdim, dtype=x.dtype, device=x.device)
    kern.moe_grouped_gemm(ys, a, w2, offsets)
    out = torch.empty_like(x)
    kern.moe_combine(out, ys, pos, w)
    return out
