"""
Custom ops. GPU tensors always go to the hand-written gfx950 HIP kernels in
``src/_C*.so`` (built by :mod:`src._build`); if that extension is missing a
GPU call raises — there is no silent eager fallback on the GPU. CPU tensors use
:mod:`src.ops.reference` (the fp32 semantics the kernels are tested against),
which lets the engine's control flow run in CPU-only tests.
"""

from __future__ import annotations

import os
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


def silu_and_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None,
                 row_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up for x = [gate | up]; row_scale (fp32 [T]): silu(r gate) * (r up) — the prefill RMSNorm
    applied after a projection of the raw residual (:func:`rms_row_scale`)."""
    if not x.is_cuda:
        if row_scale is not None:
            x = (x.float() * row_scale[:, None]).to(x.dtype)
        return ref.silu_and_mul(x)
    if out is None:
        out = torch.empty(x.shape[0], x.shape[1] // 2, dtype=x.dtype, device=x.device)
    _kern().silu_and_mul(out, x, row_scale if row_scale is not None else _empty(x.device))
    return out


def silu_and_mul_views(gate: torch.Tensor, up: torch.Tensor, out: torch.Tensor,
                       row_scale: Optional[torch.Tensor] = None, per: int = 0) -> torch.Tensor:
    """out = silu(r gate) * (r up) on [T, I] row views (unit column stride, e.g. column blocks of a wider
    buffer): the SiLU * up of one FFN column chunk, written into its columns of the [T, inter] activation.
    per: 16-byte chunks per lane (0: the launcher's choice; micro-benchmarks only)."""
    if not gate.is_cuda:
        g, u = gate.float(), up.float()
        if row_scale is not None:
            g, u = g * row_scale[:, None], u * row_scale[:, None]
        out.copy_((torch.nn.functional.silu(g) * u).to(out.dtype))
        return out
    _kern().silu_and_mul_views(out, gate, up, row_scale if row_scale is not None else _empty(gate.device), per)
    return out


def set_attn_few_pair_parts(on: bool) -> None:
    """Decode attention launch policy for few (sequence, kv head) pairs (tensor-parallel shards) at a short static
    context bound: one chunk per part, one workgroup per task (default on; off = the static split, for A/Bs)."""
    if native_available():
        _kern().attn_set_few_pair_parts(bool(on))


def rms_row_scale(resid: torch.Tensor, x: Optional[torch.Tensor], eps: float,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Prefill RMSNorm as a row scale (norm weight folded into the consuming projection): resid += x (bf16,
    in place; x None: no add) and returns rs [T] fp32 = rsqrt(mean(resid^2) + eps). The projections then run
    on the raw residual and their consumers scale the output rows (rope_and_cache / attn_prefill /
    silu_and_mul ``row_scale``): no normalised copy of the residual is written."""
    t = resid.shape[0]
    if out is None:
        out = torch.empty(t, dtype=torch.float32, device=resid.device)
    if not resid.is_cuda:
        if x is not None:
            resid.copy_((resid.float() + x.float()).to(resid.dtype))
        out.copy_(torch.rsqrt(resid.float().pow(2).mean(-1) + eps))
        return out
    _kern().rms_row_scale(out, resid, x if x is not None else _empty(resid.device), float(eps))
    return out


def rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq: int, hkv: int, head_dim: int,
                   rot_q: bool = True, row_scale: Optional[torch.Tensor] = None) -> None:
    """Rotate k (and q unless rot_q=False: prefill attention then rotates its Q rows on load, see
    attn_prefill's cos_sin) and write k / v into the paged cache. row_scale (fp32 [T], with rot_q=False):
    k and v rows are scaled by the token's RMSNorm scale (:func:`rms_row_scale`); q is left to the attention."""
    if not qkv.is_cuda:
        assert rot_q and row_scale is None, "the CPU reference path rotates q here"
        ref.rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, head_dim)
        return
    assert row_scale is None or not rot_q, "a row scale is applied with the attention's Q rotation"
    _kern().rope_and_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, head_dim, rot_q,
                           row_scale if row_scale is not None else _empty(qkv.device))


def attn_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_q_len: int, hq: int, hkv: int,
                 scale: float, out: Optional[torch.Tensor] = None, cos_sin: Optional[torch.Tensor] = None,
                 q_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Causal paged prefill attention. cos_sin ([max_pos, 128] fp32): q is NOT yet rotated, the kernel
    applies RoPE to each Q row as it loads it (token positions ctx - q_len + i). q_scale (fp32 [T], with
    cos_sin): each Q row is also scaled by its token's RMSNorm scale (:func:`rms_row_scale`)."""
    if not q.is_cuda:
        assert cos_sin is None and q_scale is None, "the CPU reference path takes a rotated q"
        return ref.attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, hq, hkv, scale).reshape(q.shape[0], -1)
    if out is None:
        out = torch.empty(q.shape[0], hq * 128, dtype=q.dtype, device=q.device)
    assert q_scale is None or cos_sin is not None, "the Q row scale is applied with the rotation"
    e = _empty(q.device)
    _kern().attn_prefill(out, q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_q_len, hq, hkv, scale,
                         cos_sin if cos_sin is not None else e, q_scale if q_scale is not None else e)
    return out


def decode_partials(max_ctx: int) -> int:
    return int(_kern().decode_partials(max_ctx))


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, max_ctx: int, hq: int, hkv: int, scale: float,
                part_o: Optional[torch.Tensor] = None, part_ml: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, counters: Optional[torch.Tensor] = None,
                merge_kernel: bool = False) -> torch.Tensor:
    """Paged decode attention. `counters` (int32, >= num_seqs * hkv, zeroed once) are the
    per-(sequence, kv head) tickets of the self-merging kernel; they are re-armed by the kernel,
    so a runner allocates them once. merge_kernel=True forces the two-launch path."""
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
    if merge_kernel:
        counters = torch.empty(0, dtype=torch.int32, device=q.device)
    elif counters is None:
        counters = torch.zeros(n * hkv, dtype=torch.int32, device=q.device)
    _kern().attn_decode(out, part_o, part_ml, counters, q, k_cache, v_cache, block_tables, ctx_lens, max_ctx, hq,
                        hkv, scale)
    return out


def attn_decode_fused(qkv_slab: torch.Tensor, ssp: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                      slot_mapping: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                      block_tables: torch.Tensor, ctx_lens: torch.Tensor, max_ctx: int, hq: int, hkv: int,
                      scale: float, eps: float, hidden: int, part_o: torch.Tensor, part_ml: torch.Tensor,
                      counters: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decode attention whose prologue does the input RMSNorm row scale (statistics ssp [T, 32],
    weight folded into Wqkv), the split-K reduction of the qkv slabs [sk, M, width], RoPE at
    position ctx-1 and the paged KV write of the new token (attention.hip, FUSED)."""
    n = ctx_lens.numel()
    if out is None:
        out = torch.empty(n, hq * 128, dtype=torch.bfloat16, device=qkv_slab.device)
    _kern().attn_decode_fused(out, part_o, part_ml, counters, qkv_slab, ssp, positions, cos_sin, slot_mapping,
                              k_cache, v_cache, block_tables, ctx_lens, max_ctx, hq, hkv, scale, eps, hidden)
    return out


def decode_advance(out, ids, pos, ctx, slots, bt, step, tokens, cnt, n_real, rows: int, block_size: int) -> None:
    """Device-side advance of the decode inputs (decode_step.hip); see ModelRunner.decode_multi."""
    _kern().decode_advance(out, ids, pos, ctx, slots, bt, step, tokens, cnt, n_real, rows, block_size)


def sample(logits, temperature=None, top_k=None, top_p=None, seeds=None, steps=None,
           out: Optional[torch.Tensor] = None, scratch=None, lm_part: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``scratch`` = (part int32 [>= rows * 32], cnt int32 [>= rows], zero): greedy rows are split over several
    workgroups each (a decode step's argmax on ~256 CUs instead of one per row); keep it for the engine's life
    (the tickets are re-armed by the kernel, so it is graph-capturable). ``lm_part`` [rows, parts, 2] int32: the
    LM head's per-column-tile candidates (:func:`linear_tiled_argmax`) — greedy rows reduce those instead."""
    if not logits.is_cuda:
        return ref.sample(logits, temperature, top_k, top_p, seeds, steps)
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    part, cnt = scratch if scratch is not None else (None, None)
    _kern().sample(out, logits, temperature, top_k, top_p, seeds, steps, part, cnt, lm_part)
    return out


def sample_advance(logits, temperature, top_k, top_p, seeds, steps, out, lm_part, ids, pos, ctx, slots, bt, tokens,
                   cnt, n_real, block_size: int, ticket, embed=None) -> torch.Tensor:
    """:func:`sample` from the LM head's candidates (``lm_part``) fused with :func:`decode_advance`: every row's
    workgroup also writes its token into the window's token row ``cnt[0]`` and advances the row's id / position /
    context / slot / step (``steps`` is read for the draw, then incremented); the last row bumps ``cnt[0]``.
    ``ticket``: int32 [1], zero, re-armed by the kernel (graph-capturable). ``embed`` = (table [V, H], h_out
    [>= rows, H], ssp_out [>= rows] fp32): also writes the next step's embedding rows of the advanced ids and their
    sums of squares, bit-identical to :func:`embed_sumsq`."""
    e = _empty(logits.device)
    table, h_out, ssp_out = embed if embed is not None else (e, e, e)
    _kern().sample_advance(out, logits, temperature, top_k, top_p, seeds, lm_part, ids, pos, ctx, slots, bt, steps,
                           tokens, cnt, n_real, block_size, ticket, table, h_out, ssp_out)
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


def gather_blocks_rows(pool: torch.Tensor, ids: torch.Tensor, dst: torch.Tensor, plane0: int, nplanes: int) -> None:
    """Planes [plane0, plane0 + nplanes) of pool blocks ``ids`` into the packet rows at device addresses ``dst``
    (int64, one per block; each row [planes, slab]) — the overlapped disaggregated export (LayerGroupExporter)."""
    _kern().gather_blocks_rows(pool, ids, dst, plane0, nplanes)


def scatter_blocks(pool: torch.Tensor, ids: torch.Tensor, buf: torch.Tensor) -> None:
    planes, nb = pool.shape[0], pool.shape[1]
    slab = pool.numel() // (planes * nb)
    if not pool.is_cuda:
        pool.view(planes, nb, slab)[:, ids.long()] = buf.view(ids.numel(), planes, slab).transpose(0, 1)
        return
    _kern().move_blocks(pool, buf, ids, False)


DECODE_GEMM_MAX_M = 128   # weight-streaming decode GEMM / fused decode path (gemm_decode.hip)
# expert-streaming grouped decode GEMM up to this many tokens (<= 128 rows per expert: 16/32/64/128-row
# images; above it: <= 128-row segments). 32 (round 1's limit) measured 14.9 vs 18.1 req/s at batch 64
MOE_DECODE_MAX_T = 128
SSP_LD = 128              # row stride of the norm-statistics arrays [tiles, SSP_LD]
SSP_MAX_TILES = 256       # statistics tiles a consumer takes at <= 32 decode rows (launchers.h)
SSP_MAX_TILES_WIDE = 128  # ... above 32 rows


def _decode_gemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.is_cuda and 1 <= x.shape[0] <= DECODE_GEMM_MAX_M and x.shape[1] % 256 == 0
            and w.shape[0] % 16 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0)


DECODE_GEMM_NT = True

def gd_tile(wr: int, kc: Optional[int] = None):
    """(weight rows, K slot) of a decode-GEMM tile. ``kc`` defaults from the legacy wr codes: 256 for
    32 / 48 / 64 rows, 128 for >= 96 rows, and odd codes 33 / 49 / 65 = the 128-wide deep-ring variants."""
    if kc is None:
        kc = 128 if (wr >= 96 or wr & 1) else 256
    return wr & ~1, kc


def gemm_decode(x: torch.Tensor, w: torch.Tensor, mode: int = 0, wr: int = 64, sk: int = 1,
                out: Optional[torch.Tensor] = None, nt: Optional[bool] = None, kc: Optional[int] = None) -> torch.Tensor:
    """Raw access to the decode GEMM kernel (see csrc/kernels/gemm_decode.hip).
    mode 0: bf16 x@w^T; mode 1: bf16 silu(gate)*up (w = [gate; up]);
    mode 2: fp32 split-K slabs [sk, M, N]. ``(wr, kc)``: the workgroup tile (:func:`gd_tile`)."""
    m = x.shape[0]
    wr, kc = gd_tile(wr, kc)
    base = mode & 31  # | 32: w pre-packed by gd_pack_weights
    n = w.shape[0] // 2 if base == 1 else w.shape[0]
    if out is None:
        if base == 2:
            out = torch.empty(sk, m, n, dtype=torch.float32, device=x.device)
        else:
            out = torch.empty(m, n, dtype=x.dtype, device=x.device)
    e = _empty(x.device)
    _kern().gemm_decode(out, x, w, mode, wr, kc, sk, DECODE_GEMM_NT if nt is None else nt, e, e, e, e, 0.0)
    return out


def gd_swizzle(r: torch.Tensor, kc: int) -> torch.Tensor:
    """16-byte chunk swizzle of LDS-image row r for a K slot of kc elements (gemm_decode.hip swz())."""
    rowb = 2 * kc
    if rowb >= 256:
        return r & 15
    if rowb == 128:
        return (r >> 1) & 7
    return (r ^ (r >> 1)) & 3


def gd_pack_weights(w: torch.Tensor, wr: int, silu: bool = False, kc: Optional[int] = None) -> torch.Tensor:
    """Re-lay a [rows, K] projection weight in the decode GEMM's tile order: for column tile t and
    K-chunk c, the tile's (wr x KC) block is contiguous and already in the kernel's LDS-image order
    (rows of the tile, 16-byte chunks XOR-swizzled by row), so every 1-KiB LDS-DMA piece is one
    linear read. silu: w = [gate; up] and a tile holds wr/2 gate rows then the matching wr/2 up
    rows. The result has w's shape (pass mode | 32 to gemm_decode)."""
    rows, k = w.shape
    wrr, kc = gd_tile(wr, kc)
    cpr = kc // 8
    no = wrr // 2 if silu else wrr
    n_out = rows // 2 if silu else rows
    assert n_out % no == 0 and k % kc == 0
    nt, nch = n_out // no, k // kc
    t = torch.arange(nt, device=w.device).view(nt, 1) * no
    j = torch.arange(no, device=w.device).view(1, no)
    idx = torch.cat([t + j, n_out + t + j], 1) if silu else (t + torch.arange(wrr, device=w.device).view(1, wrr))
    wt = w[idx.reshape(-1)].view(nt, wrr, nch, cpr, 8)
    r = torch.arange(wrr, device=w.device).view(1, wrr, 1, 1, 1)
    q = torch.arange(cpr, device=w.device).view(1, 1, 1, cpr, 1)
    sw = (q ^ gd_swizzle(r, kc)).expand(nt, wrr, nch, cpr, 8)
    wt = torch.gather(wt, 3, sw)
    return wt.permute(0, 2, 1, 3, 4).contiguous().view(rows, k)


def gd_unpack_weights(wt: torch.Tensor, wr: int, kc: Optional[int] = None) -> torch.Tensor:
    """Inverse of :func:`gd_pack_weights` (plain projections, not the SiLU pairing): the row-major weight."""
    rows, k = wt.shape
    wrr, kc = gd_tile(wr, kc)
    cpr = kc // 8
    assert rows % wrr == 0 and k % kc == 0
    nt, nch = rows // wrr, k // kc
    w = wt.view(nt, nch, wrr, cpr, 8).permute(0, 2, 1, 3, 4)
    r = torch.arange(wrr, device=wt.device).view(1, wrr, 1, 1, 1)
    q = torch.arange(cpr, device=wt.device).view(1, 1, 1, cpr, 1)
    sw = (q ^ gd_swizzle(r, kc)).expand(nt, wrr, nch, cpr, 8)  # the XOR swizzle is its own inverse
    return torch.gather(w, 3, sw).contiguous().view(rows, k)


_EMPTY: dict = {}


def _empty(dev) -> torch.Tensor:
    t = _EMPTY.get(dev)
    if t is None:
        t = _EMPTY[dev] = torch.empty(0, device=dev)
    return t


def linear_slab_residual(x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor, ssp_out: torch.Tensor,
                         counters: torch.Tensor, wr: int = 64, sk: int = 4, tiled: bool = False,
                         kc: Optional[int] = None, half_ring: bool = False) -> torch.Tensor:
    """resid += x @ w^T (bf16, in place) with split-K reduced by the last-arriving workgroup of
    each column tile, which also writes the tile's row sums of squares of the new residual to
    ssp_out [N/wr, SSP_LD] — the statistics of the next RMSNorm (whose weight is folded into the
    consuming projection). counters [N/wr] int32, zeroed once. Returns the slab scratch."""
    m, n = x.shape[0], w.shape[0]
    wr, kc = gd_tile(wr, kc)
    slab = torch.empty(sk, m, n, dtype=torch.float32, device=x.device)
    e = _empty(x.device)
    _kern().gemm_decode(slab, x, w, 3 | (32 if tiled else 0) | (64 if half_ring else 0), wr, kc, sk, DECODE_GEMM_NT,
                        resid, ssp_out, counters, e, 0.0)
    return slab


_OCC: dict = {}


def gd_occupancy(mode: int, wr: int, kc: int, sk: int, rows: int, half_ring: bool = False) -> int:
    """Resident workgroups per CU of the decode-GEMM launch these parameters select
    (hipOccupancyMaxActiveBlocksPerMultiprocessor on that instantiation; 0 off the GPU or if none exists)."""
    if not native_available() or not torch.cuda.is_available():
        return 0
    key = (mode, wr, kc, sk, rows, half_ring)
    v = _OCC.get(key)
    if v is None:
        v = max(0, int(_kern().gd_occupancy(mode | (64 if half_ring else 0), wr, kc, sk, rows, DECODE_GEMM_NT)))
        _OCC[key] = v
    return v


def linear_silu_mul_rownorm(x: torch.Tensor, w_gate_up: torch.Tensor, ssp_in: torch.Tensor, eps: float,
                            wr: Optional[int] = None, tiled: bool = False, kc: Optional[int] = None, sk: int = 1,
                            slab: Optional[torch.Tensor] = None,
                            counters: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(r * x @ gate^T) * (r * x @ up^T) with r = rsqrt(sum_t ssp_in[t] / K + eps) per row:
    RMSNorm (weight folded into w_gate_up) + gate/up + SiLU*mul in one weight stream. sk > 1 (mode 6): K
    split over sk workgroups per tile with fp32 partials in ``slab`` (>= sk * rows * 2N floats) and the tile's
    last arriver finishing (``counters``: >= N / (wr / 2) int32, zero; re-armed by the kernel)."""
    n = w_gate_up.shape[0] // 2
    if wr is None:
        wr, kc, _ = decode_tile(n, x.shape[1], 4, _bucket(x.shape[0]))
    wr, kc = gd_tile(wr, kc)
    out = torch.empty(x.shape[0], n, dtype=x.dtype, device=x.device)
    e = _empty(x.device)
    if sk > 1:
        if slab is None or counters is None:
            raise ValueError("split-K gate/up (sk > 1) needs its slab and counters")
        _kern().gemm_decode(out, x, w_gate_up, 6 | (32 if tiled else 0), wr, kc, sk, DECODE_GEMM_NT, e, slab, counters,
                            ssp_in, float(eps))
        return out
    _kern().gemm_decode(out, x, w_gate_up, 4 | (32 if tiled else 0), wr, kc, 1, DECODE_GEMM_NT, e, e, e, ssp_in,
                        float(eps))
    return out


# (N_out, K, row bucket) -> (wr, kc, sk) of the split-K gate/up (mode 6), where the full-K form's grid forces
# narrow tiles (bench/micro_gd_splitk_silu.py, profiles/micro_gd_splitk_silu_r3.jsonl): Llama-3-70B's TP=8
# shard 27.1 us vs 30.0 for the best full-K tile (32, 256). Dense 8B shapes lose with split-K (not listed).
DECODE_SILU_SPLITK_CFG = {
    (3584, 8192, 32): (64, 128, 2),   # round 4 sweep (micro_tp_tiles_r4): 26.84 us vs 30.36 for (64, 256, 2) cold
    # 64 / 128 rows (micro_tp_tiles --rows 64 / 128, profiles/micro_tp_tiles_r4_rows64_128.jsonl, cold us)
    (3584, 8192, 64): (112, 128, 4),  # 34.76 vs 41.28 for the full-K (32, 128)
    (3584, 8192, 128): (64, 128, 2),  # 46.36 vs 52.12
}


def decode_tile_silu(n: int, k: int, bucket: int = 32, row_major: bool = False):
    """(wr, kc, sk) of the norm-scaled SiLU gate/up decode GEMM: a split-K tile where one was measured faster,
    else the full-K tile (sk = 1). ``row_major``: on weights kept row-major (DECODE_TILE_CFG_RM)."""
    if row_major:
        c = DECODE_TILE_CFG_RM.get((n, k, 6, bucket)) or DECODE_TILE_CFG_RM.get((n, k, 4, bucket))
        if c is not None:
            return c
    # DIE_TILE_OVERRIDE entries with mode 6 name the split-K SiLU gate/up tile (N_out, K, 6, bucket) (in-graph A/Bs)
    c = DECODE_TILE_CFG.get((n, k, 6, bucket)) or DECODE_SILU_SPLITK_CFG.get((n, k, bucket))
    if c is not None:
        return c
    return (*decode_tile(n, k, 4, bucket)[:2], 1)


def residual_add_sumsq(resid: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """resid += x (bf16, in place); out [1, SSP_LD] = per-row sums of squares of the new residual."""
    if not x.is_cuda:
        resid.copy_((resid.float() + x.float()).to(resid.dtype))
        out.zero_()
        out[0, : x.shape[0]] = resid.float().pow(2).sum(-1)
        return out
    _kern().residual_add_sumsq(out, resid, x)
    return out


def embed_sumsq(ids: torch.Tensor, table: torch.Tensor, ssp: torch.Tensor, out: Optional[torch.Tensor] = None):
    """(table[ids] [M, H], ssp): the decode step's embedding gather and its per-row sums of squares (the first
    layer's RMSNorm statistics, ssp [1, SSP_LD]) in one launch."""
    if not table.is_cuda:
        h = torch.nn.functional.embedding(ids, table)
        if out is not None:
            h = out.copy_(h)
        return h, row_sumsq(h, out=ssp)
    h = out if out is not None else torch.empty(ids.shape[0], table.shape[1], dtype=table.dtype, device=table.device)
    _kern().embed_sumsq(h, ssp, table, ids)
    return h, ssp


def row_sumsq(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[1, SSP_LD] fp32 per-row sums of squares of x [M <= SSP_LD, H] (RMSNorm statistics)."""
    if out is None:
        out = torch.zeros(1, SSP_LD, dtype=torch.float32, device=x.device)
    if not x.is_cuda:
        out.zero_()
        out[0, : x.shape[0]] = x.float().pow(2).sum(-1)
        return out
    _kern().row_sumsq(out, x)
    return out


# (N, K, mode) -> (wr, sk), measured with bench/micro_gemm_decode.py on MI355X (cold
# weights, M = 32, nt weight loads; profiles/micro_gemm_decode_m32_r1b.jsonl). Fastest
# configs put (N/cols)*sk at (a multiple of) ~256 workgroups, one per CU.
DECODE_GEMM_CFG = {
    (6144, 4096, 2): (48, 2),      # Llama-3-8B / Mixtral qkv  (11.6 us vs hipBLASLt 15.3)
    (4096, 4096, 2): (64, 4),      # 8B o_proj                  (9.3 vs 13.3)
    (14336, 4096, 1): (112, 1),    # 8B gate/up + SiLU          (46.4 vs 53.4)
    (4096, 14336, 2): (64, 4),     # 8B down_proj               (22.2 vs 33.9)
    (128256, 4096, 0): (64, 1),    # Llama-3 LM head            (177 vs 190, 5.9 TB/s)
    (1280, 8192, 2): (64, 8),      # 70B TP=8 qkv               (7.8 vs 15.3)
    (8192, 1024, 0): (32, 1),      # 70B TP=8 o_proj            (6.3 vs 11.4)
    (3584, 8192, 1): (32, 1),      # 70B TP=8 gate/up + SiLU    (26.6 vs 29.7)
    (8192, 3584, 0): (32, 1),      # 70B TP=8 down_proj         (13.3 vs 15.6)
}
DECODE_GEMM_MAX_N = 262144
# mode 3 (split-K + last-arriver residual update), (N, K) -> (wr, sk). In isolation
# (micro_gemm_decode.py resid) wr32/sk2 wins by ~1 us, but inside the decode graph wr64/sk4
# is faster (bench decode 4.07 -> 3.93 ms/step): keep what the real step measures.
DECODE_GEMM_RESID_CFG = {
    (4096, 4096): (64, 4),     # 8B o_proj
    (4096, 14336): (64, 4),    # 8B down
}


def _cfg_for(n: int, k: int, mode: int, max_sk: int = 8):
    c = DECODE_GEMM_CFG.get((n, k, mode))
    if c is not None and c[1] <= max_sk:
        return c
    import math

    best, score = (64, 1), 1e9
    for wr in (64, 32):
        cols = wr // 2 if mode == 1 else wr
        if n % cols:
            continue
        for sk in ((1, 2, 4, 8) if mode == 2 else (1,)):
            if sk > max_sk:
                continue
            if k % (256 * sk):
                continue
            s = abs(math.log2((n // cols) * sk / 256.0))
            if s < score - 1e-9:
                best, score = (wr, sk), s
    return best


def gd_tile_valid(wr: int, kc: int, xr: int) -> bool:
    """A (wr, kc) tile has an xr-row activation image (mirror of gemm_decode.hip gd_valid)."""
    rpp = 64 // (kc // 8)
    slot = (wr + xr) * kc * 2
    s = min(8, 147456 // slot)
    per_wave = (wr + xr) // rpp // 4
    while s > 2 and (s - 1) * per_wave > 63:
        s -= 1
    red = (4 if xr < 64 and kc >= 128 else 1) * max(xr, 32) * wr * 4 + 2048
    return (s >= 2 and (wr + xr) % (4 * rpp) == 0 and xr % rpp == 0 and wr % rpp == 0
            and not (xr < 64 and kc < 128 and wr % 64) and max(s * slot, red) <= 160 * 1024)


# (N, K, mode, row bucket) -> (wr, kc, sk) for the fused decode layer's projections (mode 2 qkv slabs,
# 3 o / down residual update, 4 gate/up row-norm + SiLU), Llama-3-8B shapes, measured on MI355X with
# bench/micro_gemm_decode_large.py (cold weights, tile-order packed; profiles/micro_gemm_decode_large_r2.jsonl).
# The 32-row bucket keeps round 1's in-graph choices (DECODE_GEMM_CFG / DECODE_GEMM_RESID_CFG).
DECODE_TILE_CFG = {
    (6144, 4096, 2, 64): (96, 128, 4),     # qkv   15.0 us vs hipBLASLt 17.9
    (6144, 4096, 2, 128): (48, 128, 2),    #       20.2 vs 25.3
    (4096, 4096, 3, 64): (64, 128, 4),     # o     13.4 vs 15.3
    (4096, 4096, 3, 128): (32, 128, 2),    #       16.5 vs 24.6
    (14336, 4096, 4, 64): (112, 128, 1),   # gate/up + SiLU  45.6 vs 50.5
    (14336, 4096, 4, 128): (128, 64, 1),   #                 57.2 vs 54.7
    (4096, 14336, 3, 64): (64, 128, 4),    # down  28.3 vs 40.0
    (4096, 14336, 3, 128): (128, 64, 8),   #       38.3 vs 75.3
    # the bench's 32-row bucket, round-4 sweep (bench/micro_tp_tiles.py --shapes 8b, profiles/micro_8b_tiles_r4.jsonl,
    # cold us) confirmed in the real graph: bench 50.49 -> 51.45 req/s with all three, same box
    # (profiles/bench_r4_tile_ab.jsonl; gate/up alone 50.94, o alone 50.44)
    (4096, 4096, 3, 32): (32, 256, 2),     # o      13.96 vs 15.44 for (64, 256, 4)
    (14336, 4096, 4, 32): (128, 128, 1),   # gate/up + SiLU 42.08 vs 43.96 for (112, 128, 1)
    (4096, 14336, 3, 32): (64, 128, 4),    # down   29.6 vs 30.2 for (64, 256, 4)
    # tensor-parallel shards, 32 rows (bench/micro_tp_tiles.py, profiles/micro_tp_tiles_r4.jsonl, cold, us)
    # round 5: consumers take 256 statistics tiles at <= 32 rows, so the 70B shard's wr = 32 tiles (one workgroup
    # per CU, no split-K) are usable (bench/micro_tp_tiles.py --proj o,down, profiles/r5_tp8_tiles_wr32.jsonl):
    # o 10.00 vs 11.28 us for (64, 256, 1), down 17.20 vs 17.96 for (64, 128, 2); probe 5.74 -> 5.58 ms/step
    (8192, 1024, 3, 32): (32, 128, 1),     # 70B TP=8 o
    (8192, 3584, 3, 32): (32, 256, 1),     # 70B TP=8 down
    (4096, 2048, 3, 32): (32, 128, 2),     # 8B TP=2 o      11.48 vs 12.68
    (4096, 7168, 3, 32): (64, 128, 4),     # 8B TP=2 down   18.40 vs 18.88
    (3072, 4096, 2, 32): (48, 128, 4),     # 8B TP=2 qkv    11.08 vs 11.80
    (7168, 4096, 4, 32): (64, 128, 1),     # 8B TP=2 gate/up 24.84 vs 25.68
    (1280, 8192, 2, 64): (32, 256, 4),     # 70B TP=8 qkv at 64 rows  13.80 vs 14.40 for (32, 128, 4)
    (8192, 1024, 3, 128): (64, 64, 2),     # 70B TP=8 o at 128 rows   17.52 vs 18.20 for (64, 128, 2)
    # Llama-3-70B on ONE GPU (TP=1): decode streams the row-major weights (their tile-order copies do not fit beside
    # 141 GB); round-6 sweep (bench/micro_tp_tiles.py --shapes 70b --row-major, profiles/r6_70b_tp1_tiles.jsonl, cold us)
    (10240, 8192, 2, 32): (64, 256, 1),    # qkv            38.76 vs 43.68 for the generic (64, 256, 2)
    (28672, 8192, 4, 32): (112, 128, 1),   # gate/up + SiLU 165.76 vs 189.88 for (64, 256, 1)
    (8192, 28672, 3, 32): (128, 128, 4),   # down           80.68 vs 88.48 for (64, 256, 2)
}


def _tile_overrides(spec: str) -> dict:
    """DIE_TILE_OVERRIDE="N,K,mode,bucket=wr,kc,sk;...": decode-GEMM tiles to try in the real graph (A/B runs of
    a micro-bench winner) without editing DECODE_TILE_CFG."""
    out = {}
    for item in filter(None, (s.strip() for s in spec.split(";"))):
        key, val = item.split("=")
        out[tuple(int(v) for v in key.split(","))] = tuple(int(v) for v in val.split(","))
    return out


DECODE_TILE_CFG.update(_tile_overrides(os.environ.get("DIE_TILE_OVERRIDE", "")))
_GENERIC_TILES = ((64, 128),(128, 64), (32, 128), (64, 64), (128, 32), (64, 32), (112, 128), (96, 128), (48, 128),
                  (128, 128))


# (N, K, mode, row bucket) -> (wr, kc, sk) where the decode GEMM streams the ROW-MAJOR weights by choice
# (EngineConfig.decode_weight_layout = single: the KV pool is the constraint, no tile-order copies), measured with
# bench/micro_tp_tiles.py --row-major; shapes not listed fall back to the tile-order table's choice
# Round 6, Llama-3-8B at 32 rows: the cold sweep's row-major winners (o (64, 256, 4) 14.44 vs 15.28 us, gate/up
# (64, 256, 1) 48.28 vs 53.68, profiles/r6_8b_rm_tiles.jsonl) LOST in the graph — decode 3.96 vs 3.76 ms/step,
# profiles/r6_decode_layout_rm_tiles_negative.jsonl — so the 8B shapes keep the tile-order table's tiles.
DECODE_TILE_CFG_RM: dict = {}


def decode_tile(n: int, k: int, mode: int, bucket: int = 32, max_sk: int = 8, row_major: bool = False):
    """(wr, kc, sk) of the decode GEMM for an [N, K] projection in ``mode`` (0 bf16, 1 / 4 SiLU, 2 slabs,
    3 residual update) at steps of up to ``bucket`` rows (32, 64, 128); ``row_major``: on weights kept row-major."""
    import math

    if row_major:
        c = DECODE_TILE_CFG_RM.get((n, k, mode, bucket))
        if c is not None and c[2] <= max_sk:
            return c

    c = DECODE_TILE_CFG.get((n, k, mode, bucket))
    # mode 3 writes one statistics tile per wr columns; its consumers take at most 128 of them
    if c is not None and c[2] <= max_sk and (mode != 3 or n // c[0] <= (SSP_MAX_TILES if bucket <= 32
                                                                         else SSP_MAX_TILES_WIDE)):
        return c
    if bucket <= 32:
        if mode == 3:
            c = DECODE_GEMM_RESID_CFG.get((n, k))
            if c is None:
                wr, sk = _cfg_for(n, k, 2, max_sk)
                if wr not in (32, 64, 128) or n % wr:
                    wr = 64 if n % 64 == 0 else 32
                while sk > 1 and k % (256 * sk):
                    sk //= 2
                c = (wr, sk)
            return (*gd_tile(c[0]), c[1])
        wr, sk = _cfg_for(n, k, {4: 1}.get(mode, mode), max_sk)
        return (*gd_tile(wr), sk)
    return _generic_tile(n, k, mode, bucket, max_sk)


def _generic_tile(n: int, k: int, mode: int, bucket: int, max_sk: int = 8):
    """The (wr, kc, sk) tile that exists for `bucket` activation rows and brings the grid closest to 256
    workgroups (one per CU)."""
    import math

    best, score = None, 1e9
    for wr, kc in _GENERIC_TILES:
        cols = wr // 2 if mode in (1, 4) else wr
        if n % cols or (mode == 3 and wr not in (32, 64, 128)) or not gd_tile_valid(wr, kc, bucket):
            continue
        for sk in ((1, 2, 4, 8) if mode in (2, 3) else (1,)):
            if sk > max_sk or k % (kc * sk):
                continue
            sc = abs(math.log2((n // cols) * sk / 256.0))
            if sc < score - 1e-9:
                best, score = (wr, kc, sk), sc
    if best is None:
        raise ValueError(f"no decode-GEMM tile for N={n} K={k} mode={mode} at {bucket} rows")
    return best


def _bucket(m: int) -> int:
    return 32 if m <= 32 else (64 if m <= 64 else 128)


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w^T. Decode-sized M (<= 128 rows) runs on the weight-streaming
    gfx950 kernel (gemm_decode.hip); larger M goes to hipBLASLt."""
    if _decode_gemm_ok(x, w) and w.shape[0] % 32 == 0 and w.shape[0] <= DECODE_GEMM_MAX_N:
        wr, kc, _ = decode_tile(w.shape[0], x.shape[1], 0, _bucket(x.shape[0]))
        return gemm_decode(x, w, 0, wr, 1, out, kc=kc)
    return torch.nn.functional.linear(x, w, out=out) if out is not None else torch.nn.functional.linear(x, w)


def linear_residual(resid: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """resid += x @ w^T in place through the library GEMM's C input (beta = 1): the prefill o / down projections
    add into the residual stream in their epilogue (fp32 accumulator + bf16 C, one rounding) instead of writing
    a [T, hidden] output that a separate pass reads back with the residual. Same TN signature as
    :func:`linear`, so the prefill GEMM table's solution applies. Prefill sizes only (the decode GEMM has its
    own residual epilogue, :func:`linear_slab_residual`)."""
    return resid.addmm_(x, w.t())


def linear_tiled(x: torch.Tensor, w: torch.Tensor, wr: int, kc: int) -> torch.Tensor:
    """y = x @ w^T (bf16, decode sizes) with w packed by gd_pack_weights for the (wr, kc) tile."""
    return gemm_decode(x, w, 0 | 32, wr, 1, kc=kc)


def linear_tiled_argmax(x: torch.Tensor, w: torch.Tensor, wr: int, kc: int, amax: torch.Tensor) -> torch.Tensor:
    """linear_tiled that also writes every wr-column tile's per-row greedy candidate (max of the bf16 outputs,
    lowest column on ties) into amax [M, N / wr, 2] int32 — the LM head's share of a decode step's argmax."""
    out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
    _kern().gemm_decode_argmax(out, x, w, wr, kc, True, amax)
    return out


def linear_slab(x: torch.Tensor, w: torch.Tensor, sk: Optional[int] = None, wr: Optional[int] = None,
                tiled: bool = False, kc: Optional[int] = None) -> torch.Tensor:
    """fp32 split-K slabs [sk, M, N] of x @ w^T (decode sizes only); the
    consumer (fused_add_rms_norm_slab / rope_and_cache_slab) reduces them.
    tiled: w was packed by gd_pack_weights for this (wr, kc)."""
    if sk is None or wr is None:
        assert not tiled, "a tiled weight needs its packing wr"
        wr0, kc0, sk0 = decode_tile(w.shape[0], x.shape[1], 2, _bucket(x.shape[0]))
        wr, sk, kc = wr or wr0, sk or sk0, kc or kc0
    return gemm_decode(x, w, 2 | (32 if tiled else 0), wr, sk, kc=kc)


def linear_silu_mul(x: torch.Tensor, w_gate_up: torch.Tensor) -> torch.Tensor:
    """silu(x @ gate^T) * (x @ up^T) with w_gate_up = [gate; up] (fused epilogue
    in the decode kernel; GEMM + silu_and_mul kernel otherwise)."""
    if _decode_gemm_ok(x, w_gate_up) and (w_gate_up.shape[0] // 2) % 32 == 0:
        wr, kc, _ = decode_tile(w_gate_up.shape[0] // 2, x.shape[1], 1, _bucket(x.shape[0]))
        return gemm_decode(x, w_gate_up, 1, wr, 1, kc=kc)
    return silu_and_mul(torch.nn.functional.linear(x, w_gate_up))


def fused_add_rms_norm_slab(slab: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """residual += slab.sum(0) (bf16, in place); returns rms_norm(residual) * w."""
    if not slab.is_cuda:
        return fused_add_rms_norm(slab.sum(0).to(residual.dtype), residual, w, eps, out)
    if out is None:
        out = torch.empty(residual.shape, dtype=residual.dtype, device=residual.device)
    _kern().fused_add_rms_norm_slab(out, slab, residual, w, eps)
    return out


def rope_and_cache_slab(slab, positions, cos_sin, slot_mapping, k_cache, v_cache, hq: int, hkv: int,
                        head_dim: int, q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum the QKV split-K slabs, rotate q/k, write k/v into the paged cache;
    returns q [T, hq*D] (bf16)."""
    t = slab.shape[1]
    if q_out is None:
        q_out = torch.empty(t, hq * head_dim, dtype=torch.bfloat16, device=slab.device)
    _kern().rope_and_cache_slab(q_out, slab, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, head_dim)
    return q_out


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


def expert_parallel_local(w: torch.Tensor, ids: torch.Tensor, expert0: int, n_local: int):
    """Expert parallelism over replicated tokens: keep the (token, slot) assignments routed to the
    local experts [expert0, expert0 + n_local) (ids rebased to 0..n_local-1) and send every other
    one to a null group ``n_local`` with weight 0 — no rows are computed for it, and the TP
    all-reduce after the MoE sums the experts' contributions across ranks. Plain tensor ops: no
    host sync, hipGraph-capturable."""
    local = (ids >= expert0) & (ids < expert0 + n_local)
    ids_l = torch.where(local, ids - expert0, torch.full_like(ids, n_local))
    return torch.where(local, w, torch.zeros_like(w)), ids_l.to(ids.dtype)


MOE_ROUTE_MAX_T = 256  # fused routing for decode-sized batches; larger ones: hipBLASLt gating GEMM


def moe_route(x: torch.Tensor, router: torch.Tensor, k: int, renorm: bool = True):
    """Routing weights and expert ids [T, k] from the activations and the router weights [E, H]: one
    fused launch (logits rounded to bf16, softmax, top-k) for decode-sized GPU batches; otherwise
    the router GEMM + :func:`topk_softmax`."""
    t, e = x.shape[0], router.shape[0]
    if x.is_cuda and t <= MOE_ROUTE_MAX_T and e <= 16 and x.shape[1] % 8 == 0 and x.stride(1) == 1 \
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and router.is_contiguous() \
            and router.data_ptr() % 16 == 0:
        w = torch.empty(t, k, dtype=torch.float32, device=x.device)
        ids = torch.empty(t, k, dtype=torch.int32, device=x.device)
        _kern().moe_route(w, ids, x, router, renorm)
        return w, ids
    return topk_softmax(torch.nn.functional.linear(x, router), k, renorm)


def moe_forward_routed(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, w: torch.Tensor, ids: torch.Tensor,
                       expert0: Optional[int] = None, residual: Optional[torch.Tensor] = None,
                       ssp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """:func:`moe_forward` after routing (``w``, ``ids`` [T, k] over ALL routed experts). With
    ``residual``/``ssp``: residual += output and ssp[0, :T] = its row sums of squares (returns residual)."""
    e = w13.shape[0]
    if expert0 is not None:
        w, ids = expert_parallel_local(w, ids, expert0, e)
        return moe_apply(x, w13, w2, w, ids, e + 1, residual, ssp)
    return moe_apply(x, w13, w2, w, ids, e, residual, ssp)


def moe_forward(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, gating: torch.Tensor, k: int,
                renorm: bool = True, expert0: Optional[int] = None) -> torch.Tensor:
    """Fused-routing MoE FFN on the HIP kernels: route → align → gather →
    grouped GEMM (gate/up) → SiLU·mul → grouped GEMM (down) → weighted combine.
    No host synchronisation (hipGraph-capturable). ``expert0``: expert parallelism — ``w13``/``w2``
    hold experts [expert0, expert0 + E_local) of the ``gating.shape[1]`` routed experts, and the
    output is this rank's partial sum (see :func:`expert_parallel_local`)."""
    w, ids = topk_softmax(gating, k, renorm)
    return moe_forward_routed(x, w13, w2, w, ids, expert0)  # EP: + the null group of remote assignments


def moe_apply(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, w: torch.Tensor, ids: torch.Tensor,
              groups: int, residual: Optional[torch.Tensor] = None, ssp: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[t] = sum_j w[t, j] * expert_{ids[t, j]}(x[t]) for given routing (w [T, k] fp32, ids [T, k]
    int32). ``groups`` may exceed the number of local experts ``w13.shape[0]``: assignments to those
    extra groups are not computed (their weight must be 0)."""
    e = w13.shape[0]
    if residual is not None and not (x.is_cuda and x.shape[0] <= MOE_DECODE_MAX_T):
        return residual_add_sumsq(residual, moe_apply(x, w13, w2, w, ids, groups), ssp)
    if not x.is_cuda:
        return ref.moe_experts(x, w13, w2, w, ids)
    kern = _kern()
    t, hdim = x.shape
    k = ids.shape[1]
    inter = w13.shape[1] // 2
    ids = ids.to(torch.int32).contiguous()
    w = w.float().contiguous()
    offsets, sorted_idx, pos = moe_align(ids, groups)
    # rows of the extra groups are never computed: zero them so that weight 0 x row stays 0
    ys = (torch.zeros if groups > e else torch.empty)(t * k, hdim, dtype=x.dtype, device=x.device)
    x = x.contiguous()
    tiles = _moe_decode_tiles(hdim, inter, t)
    if tiles is not None and t <= MOE_DECODE_MAX_T:
        # decode: every expert's weights streamed once by the weight-streaming kernel, its routed
        # tokens (<= t, so the activation image of the step's row bucket holds any expert's group)
        # riding along, gathered from x by the kernel itself through the sorted order; SiLU*mul
        # fused; idle experts read nothing
        (wr1, kc1), (wr2, kc2) = tiles
        a = torch.empty(t * k, inter, dtype=x.dtype, device=x.device)
        kern.gemm_decode_grouped(a, x, w13, offsets, 1, wr1, kc1, sorted_idx, k, t, 1)
        kern.gemm_decode_grouped(ys, a, w2, offsets, 0, wr2, kc2, _NO_ROWS(x.device), 1, t, 1)
        if residual is not None:  # combine + residual add + next-norm statistics in one launch
            kern.moe_combine_residual(ssp, residual, ys, pos, w)
            return residual
        out = torch.empty_like(x)
        kern.moe_combine(out, ys, pos, w)
        return out
    seg_tiles = _moe_decode_tiles(hdim, inter, MOE_DECODE_MAX_T)
    capturing = torch.cuda.is_current_stream_capturing()
    if (t >= MOE_LIBRARY_MIN_TOKENS or seg_tiles is None) and not capturing:
        # prefill: the per-expert groups are thousands of rows — hipBLASLt GEMMs per expert at
        # ~1.5 PF/s; costs one host read of the offsets per layer
        xs = torch.empty(t * k, hdim, dtype=x.dtype, device=x.device)
        kern.moe_gather(xs, x, sorted_idx, k)
        off = offsets.tolist()
        for ei in range(e):
            a0, a1 = off[ei], off[ei + 1]
            if a1 > a0:
                act = silu_and_mul(torch.nn.functional.linear(xs[a0:a1], w13[ei]))
                torch.nn.functional.linear(act, w2[ei], out=ys[a0:a1])
    else:
        # between the decode path and the library path (and under graph capture): the expert-streaming
        # grouped GEMM with each expert's rows cut into segments of <= 128 (offsets built on the device,
        # no host read); an expert with r rows streams its weights ceil(r / 128) times
        if seg_tiles is None:
            raise ValueError(f"MoE shapes hidden={hdim} inter={inter} do not tile the grouped decode GEMM "
                             "(needed under graph capture)")
        (wr1, kc1), (wr2, kc2) = seg_tiles
        segs = (t + MOE_DECODE_MAX_T - 1) // MOE_DECODE_MAX_T
        j = torch.arange(segs, device=x.device, dtype=torch.int32) * MOE_DECODE_MAX_T
        off_v = torch.minimum(offsets[:-1, None] + j[None, :], offsets[1:, None]).reshape(-1)
        off_v = torch.cat([off_v, offsets[-1:]]).to(torch.int32).contiguous()
        a = torch.empty(t * k, inter, dtype=x.dtype, device=x.device)
        kern.gemm_decode_grouped(a, x, w13, off_v, 1, wr1, kc1, sorted_idx, k, MOE_DECODE_MAX_T, segs)
        kern.gemm_decode_grouped(ys, a, w2, off_v, 0, wr2, kc2, _NO_ROWS(x.device), 1, MOE_DECODE_MAX_T, segs)
    out = torch.empty_like(x)
    kern.moe_combine(out, ys, pos, w)
    if residual is not None:
        return residual_add_sumsq(residual, out, ssp)
    return out


MOE_LIBRARY_MIN_TOKENS = 256
_NO_ROWS_CACHE: dict = {}


def _NO_ROWS(device) -> torch.Tensor:
    """Empty int32 tensor: 'no gather' for gemm_decode_grouped (cached per device, graph-safe)."""
    t = _NO_ROWS_CACHE.get(device)
    if t is None:
        t = _NO_ROWS_CACHE[device] = torch.empty(0, dtype=torch.int32, device=device)
    return t


def _moe_decode_tiles(hdim: int, inter: int, t: int):
    """((wr, kc) of the gate/up grouped GEMM, (wr, kc) of the down one) for a decode step of t tokens, or
    None when the shapes do not tile. Up to 32 rows: round 1's measured choice (gate/up as the dense
    gate/up shape, down wr 64 / 32 at a 256-wide K slot); above, the row bucket's generic tile."""
    if hdim % 32 or inter % 32:
        return None
    if t <= 32:
        wr1 = _cfg_for(inter, hdim, 1)[0]
        if not (hdim % 256 or inter % 256 or inter % (wr1 // 2) or hdim % 64):
            return gd_tile(wr1), gd_tile(64)
    try:  # the row bucket's generic tiles (also for small shards, e.g. experts split under TP)
        b = _bucket(t)
        wr1, kc1, _ = _generic_tile(inter, hdim, 1, b, max_sk=1)
        wr2, kc2, _ = _generic_tile(hdim, inter, 0, b, max_sk=1)
    except ValueError:
        return None
    return (wr1, kc1), (wr2, kc2)


def _moe_down_wr(hdim: int, inter: int) -> int:
    return 64 if hdim % 64 == 0 else 32
