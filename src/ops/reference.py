"""
Plain-PyTorch fp32 reference implementations of every custom op.

They define the semantics the gfx950 kernels must match (the numerics tests
compare kernel vs. these) and run the engine on CPU tensors for control-flow
tests. They are never used for GPU tensors: :mod:`src.ops` routes GPU tensors
to the HIP extension and raises if it is missing.
"""

from __future__ import annotations

import math
from typing import Optional

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    r = (x.float() + residual.float()).to(residual.dtype)
    return rms_norm(r, w, eps), r


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    i = x.shape[-1] // 2
    g, u = x[..., :i].float(), x[..., i:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None, scaling: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: cos in the first half, sin in the second."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) / half))
    if scaling and scaling.get("rope_type") == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * math.pi / inv
        lo_w, hi_w = old / lo, old / hi
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_w, inv / factor, inv)
        mid = (wavelen <= lo_w) & (wavelen >= hi_w)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] neox-style rotation."""
    d = x.shape[-1]
    half = d // 2
    cs = cos_sin[positions.long()]
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    xf = x.float()
    a, b = xf[..., :half], xf[..., half:]
    return torch.cat([a * cos - b * sin, b * cos + a * sin], dim=-1).to(x.dtype)


def rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, head_dim):
    t = qkv.shape[0]
    q = qkv[:, : hq * head_dim].view(t, hq, head_dim)
    k = qkv[:, hq * head_dim:(hq + hkv) * head_dim].view(t, hkv, head_dim)
    v = qkv[:, (hq + hkv) * head_dim:(hq + 2 * hkv) * head_dim].view(t, hkv, head_dim)
    qr = apply_rope(q, positions, cos_sin)
    kr = apply_rope(k, positions, cos_sin)
    qkv[:, : hq * head_dim] = qr.reshape(t, -1)
    bs = k_cache.shape[2]
    for i in range(t):
        s = int(slot_mapping[i])
        if s < 0:
            continue
        k_cache[s // bs, :, s % bs] = kr[i]
        v_cache[s // bs, :, s % bs] = v[i]


def gather_kv(cache: torch.Tensor, block_table: torch.Tensor, n: int) -> torch.Tensor:
    """[n, hkv, D] rows 0..n-1 of one sequence from the paged cache."""
    bs = cache.shape[2]
    pos = torch.arange(n, device=cache.device)
    blocks = block_table[(pos // bs).long()].long()
    return cache[blocks, :, pos % bs]


def attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, hq, hkv, scale):
    """Causal paged attention; q [T, >=hq*D] (rows may be strided) → [T, hq, D]."""
    d = 128
    out = torch.empty(q.shape[0], hq, d, dtype=q.dtype, device=q.device)
    g = hq // hkv
    for s in range(ctx_lens.numel()):
        a, b = int(cu_q[s]), int(cu_q[s + 1])
        qlen, ctx = b - a, int(ctx_lens[s])
        if qlen == 0:
            continue
        qs = q[a:b, : hq * d].reshape(qlen, hq, d).float()
        k = gather_kv(k_cache, block_tables[s], ctx).float().repeat_interleave(g, dim=1)
        v = gather_kv(v_cache, block_tables[s], ctx).float().repeat_interleave(g, dim=1)
        sc = torch.einsum("qhd,khd->hqk", qs, k) * scale
        qpos = torch.arange(ctx - qlen, ctx, device=q.device)[:, None]
        kpos = torch.arange(ctx, device=q.device)[None, :]
        sc = sc.masked_fill((kpos > qpos)[None], float("-inf"))
        p = torch.softmax(sc, dim=-1)
        out[a:b] = torch.einsum("hqk,khd->qhd", p, v).to(q.dtype)
    return out


def sample(logits, temperature=None, top_k=None, top_p=None, seeds=None, steps=None):
    """Greedy where temperature==0; otherwise a (non-bit-exact) torch sampler
    with the same filtering semantics (top-k, then top-p on the renormalised set)."""
    out = torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    for r in range(logits.shape[0]):
        row = logits[r].float()
        t = float(temperature[r]) if temperature is not None else 0.0
        k = int(top_k[r]) if top_k is not None else 0
        if t <= 0 or k == 1:
            out[r] = int(torch.argmax(row))
            continue
        z = row / t
        keep = torch.ones_like(z, dtype=torch.bool)
        if 0 < k < z.numel():
            kth = torch.topk(z, k).values[-1]
            keep &= z >= kth
        p = float(top_p[r]) if top_p is not None else 1.0
        if p < 1.0:
            zz = z.masked_fill(~keep, float("-inf"))
            probs = torch.softmax(zz, -1)
            sp, si = torch.sort(probs, descending=True)
            cum = torch.cumsum(sp, 0)
            cut = int(torch.searchsorted(cum, torch.tensor(p, device=cum.device))) + 1
            thr = sp[min(cut, sp.numel()) - 1]
            keep &= probs >= thr
        probs = torch.softmax(z.masked_fill(~keep, float("-inf")), -1)
        gen = torch.Generator(device="cpu")
        gen.manual_seed(int(seeds[r]) * 1000003 + int(steps[r]) if seeds is not None and steps is not None else 0)
        out[r] = int(torch.multinomial(probs.cpu(), 1, generator=gen))
    return out


def topk_softmax(gating: torch.Tensor, k: int, renorm: bool = True):
    p = torch.softmax(gating.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return w, ids.int()


def moe_forward(x, w13, w2, gating, k: int, renorm: bool = True):
    """Reference MoE FFN: x [T,H], w13 [E, 2I, H], w2 [E, H, I]."""
    w, ids = topk_softmax(gating, k, renorm)
    return moe_experts(x, w13, w2, w, ids)


def moe_experts(x, w13, w2, w, ids):
    """Experts' weighted sum for given routing (w [T,k], ids [T,k]); ids >= E are skipped."""
    out = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
    inter = w2.shape[-1]
    for e in range(w13.shape[0]):
        tok, slot = (ids == e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        h = x[tok].float() @ w13[e].float().t()
        a = torch.nn.functional.silu(h[:, :inter]) * h[:, inter:]
        y = a.to(x.dtype).float() @ w2[e].float().t()
        out.index_add_(0, tok, y * w[tok, slot][:, None])
    return out.to(x.dtype)
