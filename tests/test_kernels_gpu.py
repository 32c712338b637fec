"""Numerics of every hand-written gfx950 kernel against the plain PyTorch fp32
reference of the same op (src/ops/reference.py). GPU only."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from src import ops  # noqa: E402
from src.ops import reference as ref  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert ops.native_available(), "HIP extension must be built for GPU tests"
    torch.manual_seed(0)
    return torch.device("cuda:0")


def close(a, b, atol, rtol=0.0):
    d = (a.float() - b.float()).abs()
    lim = atol + rtol * b.float().abs()
    bad = (d > lim).sum().item()
    assert bad == 0, f"{bad} elements off; max abs err {d.max().item():.4g}"


@pytest.mark.parametrize("hidden", [4096, 8192, 1024])
def test_rms_norm(dev, hidden):
    x = torch.randn(37, hidden, device=dev, dtype=torch.bfloat16)
    w = torch.randn(hidden, device=dev, dtype=torch.bfloat16)
    close(ops.rms_norm(x, w, 1e-5), ref.rms_norm(x, w, 1e-5), atol=2e-2, rtol=1e-2)


def test_rms_norm_strided_input(dev):
    big = torch.randn(9, 6144, device=dev, dtype=torch.bfloat16)
    x = big[:, :4096]
    w = torch.randn(4096, device=dev, dtype=torch.bfloat16)
    close(ops.rms_norm(x, w, 1e-5), ref.rms_norm(x.contiguous(), w, 1e-5), atol=2e-2, rtol=1e-2)


def test_fused_add_rms_norm(dev):
    x = torch.randn(33, 4096, device=dev, dtype=torch.bfloat16)
    r = torch.randn(33, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.randn(4096, device=dev, dtype=torch.bfloat16)
    y_ref, r_ref = ref.fused_add_rms_norm(x, r.clone(), w, 1e-5)
    r2 = r.clone()
    y = ops.fused_add_rms_norm(x, r2, w, 1e-5)
    close(r2, r_ref, atol=1e-2, rtol=1e-2)
    close(y, y_ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("inter", [14336, 3584, 64])
def test_silu_and_mul(dev, inter):
    x = torch.randn(19, 2 * inter, device=dev, dtype=torch.bfloat16)
    close(ops.silu_and_mul(x), ref.silu_and_mul(x), atol=2e-2, rtol=1e-2)


def _paged(num_blocks, hkv, bs, dev):
    k = torch.zeros(num_blocks, hkv, bs, 128, device=dev, dtype=torch.bfloat16)
    return k, torch.zeros_like(k)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 1), (16, 16)])
def test_rope_and_cache(dev, hq, hkv):
    t, bs, nb = 45, 16, 16
    qkv = torch.randn(t, (hq + 2 * hkv) * 128, device=dev, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (t,), device=dev)
    slots = torch.randperm(nb * bs, device=dev)[:t]
    slots[3] = -1
    cs = ref.rope_cos_sin(4096, 128, 500000.0, dev)
    kc, vc = _paged(nb, hkv, bs, dev)
    kr, vr = _paged(nb, hkv, bs, dev)
    q1 = qkv.clone()
    q2 = qkv.clone()
    ops.rope_and_cache(q1, pos, cs, slots, kc, vc, hq, hkv, 128)
    ref.rope_and_cache(q2, pos.cpu(), cs, slots.cpu(), kr, vr, hq, hkv, 128)
    close(q1, q2, atol=2e-2, rtol=1e-2)
    close(kc, kr, atol=2e-2, rtol=1e-2)
    close(vc, vr, atol=0)


def _make_seqs(qlens, ctxs, hkv, bs, dev, g):
    hq = hkv * g
    nseq = len(qlens)
    max_blocks = max((c + bs - 1) // bs for c in ctxs) + 1
    total = sum((c + bs - 1) // bs for c in ctxs) + 4
    perm = torch.randperm(total).tolist()
    bt = torch.zeros(nseq, max_blocks, dtype=torch.int32)
    p = 0
    for i, c in enumerate(ctxs):
        nb = (c + bs - 1) // bs
        bt[i, :nb] = torch.tensor(perm[p:p + nb], dtype=torch.int32)
        p += nb
    kc = torch.randn(total, hkv, bs, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(total, hkv, bs, 128, device=dev, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0).tolist()), dtype=torch.int32)
    t = int(cu[-1])
    # q rows embedded in a wider qkv-like buffer (strided rows, as in the model)
    qkv = torch.randn(t, (hq + 2 * hkv) * 128, device=dev, dtype=torch.bfloat16)
    q = qkv[:, : hq * 128]
    return q, kc, vc, bt.to(dev), cu.to(dev), torch.tensor(ctxs, dtype=torch.int32, device=dev), hq


@pytest.mark.parametrize("g", [4, 8, 1])
def test_attn_prefill(dev, g):
    hkv = 8 if g != 8 else 1
    if g == 1:
        hkv = 4
    qlens = [1, 37, 128, 200, 64]
    ctxs = [1, 37, 300, 200, 1000]          # ctx > qlen: chunked prefill over cached prefix
    q, kc, vc, bt, cu, ctx, hq = _make_seqs(qlens, ctxs, hkv, 16, dev, g)
    scale = 1 / math.sqrt(128)
    out = ops.attn_prefill(q, kc, vc, bt, cu, ctx, max(qlens), hq, hkv, scale)
    r = ref.attention(q, kc, vc, bt, cu, ctx, hq, hkv, scale).reshape(q.shape[0], -1)
    close(out, r, atol=2.5e-2, rtol=2e-2)


@pytest.mark.parametrize("g", [4, 8])
def test_attn_prefill_fused_rope(dev, g):
    """Prefill attention that rotates its Q rows on load (cos_sin) == RoPE applied to q first, and the
    fp32 reference on the rotated q; positions ctx - q_len + i (chunked prefill over a cached prefix)."""
    hkv = 8 if g == 4 else 1
    qlens = [1, 37, 128, 200, 64]
    ctxs = [1, 37, 300, 200, 1000]
    q, kc, vc, bt, cu, ctx, hq = _make_seqs(qlens, ctxs, hkv, 16, dev, g)
    cs = ref.rope_cos_sin(4096, 128, 500000.0, dev)
    pos = torch.cat([torch.arange(c - n, c) for n, c in zip(qlens, ctxs)]).to(dev)
    # q rotated up front in fp32 (the rope kernel's math), rounded to bf16 as the unfused path stores it
    qr32 = q.float().view(q.shape[0], hq, 128)
    co, si = cs[pos, :64][:, None, :], cs[pos, 64:][:, None, :]
    a, b = qr32[..., :64], qr32[..., 64:]
    qr = torch.cat([a * co - b * si, b * co + a * si], -1).to(torch.bfloat16).view_as(q)
    scale = 1 / math.sqrt(128)
    fused = ops.attn_prefill(q, kc, vc, bt, cu, ctx, max(qlens), hq, hkv, scale, cos_sin=cs)
    plain = ops.attn_prefill(qr, kc, vc, bt, cu, ctx, max(qlens), hq, hkv, scale)
    close(fused, plain, atol=1e-2, rtol=1e-2)
    r = ref.attention(qr, kc, vc, bt, cu, ctx, hq, hkv, scale).reshape(q.shape[0], -1)
    close(fused, r, atol=2.5e-2, rtol=2e-2)


@pytest.mark.parametrize("nseq,plen", [(32, 512), (4, 4096), (1, 8192)])
def test_attn_prefill_served_lengths(dev, nseq, plen):
    """The exact configuration behind the headline and the long-prompt rows: Llama-3-8B
    heads (32 q / 8 kv), whole-prompt causal prefill of nseq x plen tokens with RoPE fused into the Q load,
    the XCD-aware workgroup order, 8-wave workgroups and lazy rescale — against the fp32 reference on the
    pre-rotated q, computed on the GPU."""
    g, hkv = 4, 8
    torch.manual_seed(1000 + plen)
    q, kc, vc, bt, cu, ctx, hq = _make_seqs([plen] * nseq, [plen] * nseq, hkv, 16, dev, g)
    cs = ref.rope_cos_sin(8192, 128, 500000.0, dev)
    pos = torch.cat([torch.arange(plen)] * nseq).to(dev)
    qr32 = q.float().view(q.shape[0], hq, 128)
    co, si = cs[pos, :64][:, None, :], cs[pos, 64:][:, None, :]
    a, b = qr32[..., :64], qr32[..., 64:]
    qr = torch.cat([a * co - b * si, b * co + a * si], -1).to(torch.bfloat16).view_as(q)
    del qr32, a, b
    scale = 1 / math.sqrt(128)
    fused = ops.attn_prefill(q, kc, vc, bt, cu, ctx, plen, hq, hkv, scale, cos_sin=cs)
    r = ref.attention(qr, kc, vc, bt, cu, ctx, hq, hkv, scale).reshape(q.shape[0], -1)
    close(fused, r, atol=2.5e-2, rtol=2e-2)
    # and relative error over the whole output (a structured error would show here first)
    err = float((fused.float() - r.float()).norm() / r.float().norm())
    assert err < 1e-2, err


def test_rope_and_cache_keeps_q(dev):
    """rot_q=False: k rotated and cached exactly as with rot_q=True, q left untouched."""
    hq, hkv, t, bs, nb = 32, 8, 45, 16, 16
    qkv = torch.randn(t, (hq + 2 * hkv) * 128, device=dev, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (t,), device=dev)
    slots = torch.randperm(nb * bs, device=dev)[:t]
    cs = ref.rope_cos_sin(4096, 128, 500000.0, dev)
    kc1, vc1 = _paged(nb, hkv, bs, dev)
    kc2, vc2 = _paged(nb, hkv, bs, dev)
    q1, q2 = qkv.clone(), qkv.clone()
    ops.rope_and_cache(q1, pos, cs, slots, kc1, vc1, hq, hkv, 128)
    ops.rope_and_cache(q2, pos, cs, slots, kc2, vc2, hq, hkv, 128, rot_q=False)
    assert torch.equal(q2[:, : hq * 128], qkv[:, : hq * 128])
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2)


# ---------------------------------------------------------------- prefill RMSNorm as a row scale
@pytest.mark.parametrize("t,h,add", [(700, 4096, True), (300, 8192, True), (129, 4096, False), (5, 1024, True)])
def test_rms_row_scale(dev, t, h, add):
    """resid += x (bf16) and rs = rsqrt(mean(resid^2) + eps) of the rounded residual, against fp32."""
    res = torch.randn(t, h, device=dev, dtype=torch.bfloat16) * 3
    x = torch.randn(t, h, device=dev, dtype=torch.bfloat16) if add else None
    expect = (res.float() + x.float()).to(torch.bfloat16) if add else res.clone()
    rs = ops.rms_row_scale(res, x, 1e-5)
    assert torch.equal(res, expect)
    close(rs, torch.rsqrt(expect.float().pow(2).mean(-1) + 1e-5), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("t,n,k", [(2048, 4096, 4096), (300, 4096, 14336), (129, 1024, 512)])
def test_linear_residual(dev, t, n, k):
    """Prefill o / down with the residual add in the GEMM epilogue (beta = 1, in place) against fp32
    resid + x @ w^T, rounded once."""
    res = torch.randn(t, n, device=dev, dtype=torch.bfloat16) * 2
    x = torch.randn(t, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    want = res.float() + x.float() @ w.float().t()
    ptr = res.data_ptr()
    out = ops.linear_residual(res, x, w)
    assert out.data_ptr() == ptr == res.data_ptr()
    close(res, want, atol=2e-2, rtol=1e-2)


def test_prefill_gemm_residual_matches_norm_pass_add(dev):
    """llama-mini prefill (> 128 tokens: the row-scale path): o / down added in the GEMM epilogue vs written out
    and added by the norm pass — the same hidden states and KV up to one bf16 rounding per add."""
    from src.models.llama import AttnMetadata, CausalLM
    from src.models.presets import get_preset

    m = CausalLM(get_preset("llama-mini"), "cuda:0", seed=3, max_position=4096, full_init=True)
    assert m.norms_folded
    t = 4096
    nb = (t + 15) // 16
    g = torch.Generator(device="cuda:0").manual_seed(1)
    ids = torch.randint(3, 32000, (t,), device=dev, generator=g)
    pos = torch.arange(t, device=dev)
    hidden, pools = {}, {}
    for key, resid in (("epilogue", True), ("norm_pass", False)):
        m.prefill_gemm_residual = resid
        pool = torch.zeros(m.arch.num_layers, 2, nb, m.hkv, 16, 128, dtype=m.dtype, device=dev)
        meta = AttnMetadata(True, pos.clone(), torch.arange(nb, dtype=torch.int32, device=dev)[None],
                            torch.tensor([t], dtype=torch.int32, device=dev),
                            torch.tensor([0, t], dtype=torch.int32, device=dev), t)
        assert m._prefill_row_scale(torch.empty(t, 1, device=dev), meta)
        hidden[key], pools[key] = m.forward(ids, pos, meta, pool).float(), pool.float()
    torch.cuda.synchronize()
    m.prefill_gemm_residual = True
    # layer 0's K / V come before any residual add: identical; later layers and the output within bf16 noise
    for key in ("norm_pass",):
        assert torch.equal(pools["epilogue"][0], pools[key][0])
        close(pools[key], pools["epilogue"], atol=6e-2, rtol=5e-2)
        close(hidden[key], hidden["epilogue"], atol=8e-2, rtol=5e-2)
        rel = (hidden[key] - hidden["epilogue"]).norm() / hidden["epilogue"].norm()
        assert rel < 2e-2, (key, rel)


def test_silu_and_mul_row_scale(dev):
    t, inter = 37, 3584
    x = torch.randn(t, 2 * inter, device=dev, dtype=torch.bfloat16) * 4
    rs = torch.rand(t, device=dev) + 0.1
    xs = x.float() * rs[:, None]
    r = torch.nn.functional.silu(xs[:, :inter]) * xs[:, inter:]
    close(ops.silu_and_mul(x, row_scale=rs), r, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("per", [0, 1, 3, 7, 8])
@pytest.mark.parametrize("inter,blocks", [(14336, 2), (7168, 1), (1008, 2), (64, 1)])
def test_silu_and_mul_views(dev, per, inter, blocks):
    """SiLU * up of FFN column blocks: gate / up are the two halves of each block's [T, 2c] GEMM output, the
    result goes into the block's columns of a wider [T, inter] activation (strided rows on both sides), at
    every chunks-per-lane count; the same bits as the [gate | up] layout's default launch."""
    t, c = 29, inter // blocks
    x = torch.randn(t, 2 * inter, device=dev, dtype=torch.bfloat16) * 3
    rs = torch.rand(t, device=dev) + 0.25
    want = ops.silu_and_mul(x, row_scale=rs)
    xs = x.float() * rs[:, None]
    close(want, torch.nn.functional.silu(xs[:, :inter]) * xs[:, inter:], atol=3e-2, rtol=2e-2)
    # the same columns re-laid as blocks [gate_i | up_i] of width 2c
    blk = torch.cat([torch.cat([x[:, c * i:c * (i + 1)], x[:, inter + c * i:inter + c * (i + 1)]], 1)
                     for i in range(blocks)], 1)
    out = torch.full((t, inter + 8), 7.0, device=dev, dtype=torch.bfloat16)  # wider rows, 8 guard columns
    for i in range(blocks):
        y = blk[:, 2 * c * i:2 * c * (i + 1)]
        ops.silu_and_mul_views(y[:, :c], y[:, c:], out[:, c * i:c * (i + 1)], rs, per=per)
    assert torch.equal(out[:, :inter], want)
    assert bool((out[:, inter:] == 7).all())


def test_rope_and_cache_row_scale(dev):
    """row_scale: k (rotated) and v are cached scaled by the token's factor; q stays untouched."""
    hq, hkv, t, bs, nb = 32, 8, 45, 16, 16
    qkv = torch.randn(t, (hq + 2 * hkv) * 128, device=dev, dtype=torch.bfloat16)
    rs = torch.rand(t, device=dev) + 0.25
    pos = torch.randint(0, 4000, (t,), device=dev)
    slots = torch.randperm(nb * bs, device=dev)[:t]
    cs = ref.rope_cos_sin(4096, 128, 500000.0, dev)
    kc1, vc1 = _paged(nb, hkv, bs, dev)
    kc2, vc2 = _paged(nb, hkv, bs, dev)
    scaled = qkv.float()
    scaled[:, hq * 128:] *= rs[:, None]
    q1, q2 = scaled.to(torch.bfloat16), qkv.clone()
    ops.rope_and_cache(q1, pos, cs, slots, kc1, vc1, hq, hkv, 128, rot_q=False)
    ops.rope_and_cache(q2, pos, cs, slots, kc2, vc2, hq, hkv, 128, rot_q=False, row_scale=rs)
    assert torch.equal(q2[:, : hq * 128], qkv[:, : hq * 128])
    close(kc2, kc1, atol=2e-2, rtol=1e-2)
    close(vc2, vc1, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("g", [4, 8])
def test_attn_prefill_q_scale(dev, g):
    """q_scale: the Q rows are scaled by their token's factor together with the rotation on load — the same as
    attention over the pre-scaled q."""
    hkv = 8 if g == 4 else 1
    qlens = [1, 37, 128, 200, 64]
    ctxs = [1, 37, 300, 200, 1000]
    q, kc, vc, bt, cu, ctx, hq = _make_seqs(qlens, ctxs, hkv, 16, dev, g)
    cs = ref.rope_cos_sin(4096, 128, 500000.0, dev)
    rs = torch.rand(q.shape[0], device=dev) + 0.25
    qs = (q.float() * rs[:, None]).to(torch.bfloat16)
    scale = 1 / math.sqrt(128)
    a = ops.attn_prefill(q, kc, vc, bt, cu, ctx, max(qlens), hq, hkv, scale, cos_sin=cs, q_scale=rs)
    b = ops.attn_prefill(qs, kc, vc, bt, cu, ctx, max(qlens), hq, hkv, scale, cos_sin=cs)
    close(a, b, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("g,bs,merge", [(4, 16, False), (8, 16, False), (4, 32, False), (1, 16, False),
                                         (2, 16, False), (4, 16, True)])
def test_attn_decode(dev, g, bs, merge):
    hkv = 8 if g == 4 else (1 if g == 8 else 4)
    ctxs = [1, 17, 64, 65, 300, 1000, 2049]   # one-part pairs (direct output) and multi-part pairs (ticket merge)
    q, kc, vc, bt, _, ctx, hq = _make_seqs([1] * len(ctxs), ctxs, hkv, bs, dev, g)
    scale = 1 / math.sqrt(128)
    max_ctx = 4096
    bt_wide = torch.zeros(bt.shape[0], max_ctx // bs, dtype=torch.int32, device=dev)
    bt_wide[:, : bt.shape[1]] = bt
    cnt = torch.zeros(len(ctxs) * hkv, dtype=torch.int32, device=dev)
    out = ops.attn_decode(q, kc, vc, bt_wide, ctx, max_ctx, hq, hkv, scale, counters=cnt, merge_kernel=merge)
    cu = torch.arange(len(ctxs) + 1, dtype=torch.int32, device=dev)
    r = ref.attention(q, kc, vc, bt, cu, ctx, hq, hkv, scale).reshape(q.shape[0], -1)
    close(out, r, atol=2.5e-2, rtol=2e-2)
    # the merge tickets are re-armed: a second launch on the same counters gives the same answer
    out2 = ops.attn_decode(q, kc, vc, bt_wide, ctx, max_ctx, hq, hkv, scale, counters=cnt, merge_kernel=merge)
    assert torch.equal(out, out2)
    assert int(cnt.abs().sum()) == 0


def test_attn_decode_batch32(dev):
    """The serving shape: 32 sequences x 8 kv heads (one task per CU, no partials), plus a
    single long sequence (every CU on one pair, all-partials merge)."""
    hkv, g = 8, 4
    scale = 1 / math.sqrt(128)
    # the mixed list has one-chunk contexts and chunk boundaries; a single long sequence takes the
    # static split with every part merged by the last arriver
    mixed = [1, 17, 64, 65, 127, 128, 129] + [300 + 37 * i for i in range(25)]
    for ctxs in ([512 + 7 * i for i in range(32)], mixed, [8000]):
        q, kc, vc, bt, _, ctx, hq = _make_seqs([1] * len(ctxs), ctxs, hkv, 16, dev, g)
        bt_wide = torch.zeros(bt.shape[0], 8192 // 16, dtype=torch.int32, device=dev)
        bt_wide[:, : bt.shape[1]] = bt
        cnt = torch.zeros(len(ctxs) * hkv, dtype=torch.int32, device=dev)
        out = ops.attn_decode(q, kc, vc, bt_wide, ctx, 8192, hq, hkv, scale, counters=cnt)
        cu = torch.arange(len(ctxs) + 1, dtype=torch.int32, device=dev)
        r = ref.attention(q, kc, vc, bt, cu, ctx, hq, hkv, scale).reshape(q.shape[0], -1)
        close(out, r, atol=2.5e-2, rtol=2e-2)
        out2 = ops.attn_decode(q, kc, vc, bt_wide, ctx, 8192, hq, hkv, scale, counters=cnt)
        assert torch.equal(out, out2) and int(cnt.abs().sum()) == 0  # tickets re-armed


def test_attn_softmax_spike(dev):
    """Force the online-softmax rescale branch: one key with a huge score late in the sequence."""
    g, hkv = 4, 2
    q, kc, vc, bt, cu, ctx, hq = _make_seqs([100], [700], hkv, 16, dev, g)
    # make key 650 align strongly with every query of head group 0
    blk, off = bt[0, 650 // 16].item(), 650 % 16
    kc[blk, 0, off] = (q[0, :128].float() * 8).to(torch.bfloat16)
    scale = 1 / math.sqrt(128)
    out = ops.attn_prefill(q, kc, vc, bt, cu, ctx, 100, hq, hkv, scale)
    r = ref.attention(q, kc, vc, bt, cu, ctx, hq, hkv, scale).reshape(q.shape[0], -1)
    close(out, r, atol=3e-2, rtol=2e-2)
    bt_wide = torch.zeros(1, 256, dtype=torch.int32, device=dev)
    bt_wide[:, : bt.shape[1]] = bt
    ctx1 = torch.tensor([700], dtype=torch.int32, device=dev)
    qd = q[99:100]
    out_d = ops.attn_decode(qd, kc, vc, bt_wide, ctx1, 4096, hq, hkv, scale)
    close(out_d, r[99:100], atol=3e-2, rtol=2e-2)


def test_sampling_greedy_and_filters(dev):
    v = 128256
    logits = torch.randn(6, v, device=dev, dtype=torch.bfloat16) * 3
    out = ops.sample(logits)
    assert torch.equal(out.cpu(), logits.float().argmax(-1).cpu())
    # the batched argmax pass at vocabularies below / between its load batches, ties to the lowest index,
    # and an all -inf row (-> token 0, never an out-of-range id)
    for vs in (8, 1000, 8192 * 8 + 8):
        lg = (torch.randn(3, vs, device=dev) * 3).to(torch.bfloat16)
        lg[1, vs // 2] = lg[1, vs - 1] = 100.0
        lg[2] = float("-inf")
        got = ops.sample(lg).cpu()
        want = lg.float().argmax(-1).cpu()
        assert got[0] == want[0] and got[1] == vs // 2 and got[2] == 0, (vs, got, want)
    temp = torch.full((6,), 0.8, device=dev)
    topk = torch.tensor([1, 5, 5, 0, 0, 50], dtype=torch.int32, device=dev)
    topp = torch.tensor([1.0, 1.0, 0.5, 1e-6, 0.9, 0.9], device=dev)
    seeds = torch.arange(6, device=dev, dtype=torch.long)
    top5 = torch.topk(logits.float(), 5, -1).indices.cpu()
    for step in range(20):
        steps = torch.full((6,), step, device=dev, dtype=torch.long)
        s = ops.sample(logits, temp, topk, topp, seeds, steps).cpu()
        # bf16 logits tie often at the top (spacing 1/16 near 12): compare values, not indices
        lc = logits.float().cpu()
        assert lc[0, s[0]] == lc[0].max()         # top_k = 1 → greedy
        assert lc[1, s[1]] >= lc[1, top5[1, 4]] and lc[2, s[2]] >= lc[2, top5[2, 4]]
        assert lc[3, s[3]] == lc[3].max()         # tiny top_p → argmax
    # reproducible per (seed, step)
    a = ops.sample(logits, temp, topk, topp, seeds, steps)
    b = ops.sample(logits, temp, topk, topp, seeds, steps)
    assert torch.equal(a, b)


def test_sampling_split_greedy_argmax(dev):
    """The split greedy argmax (ops.sample with scratch: each greedy row argmax'ed by up to 16 workgroups whose
    slice winners the last arriver combines) equals torch's argmax at 1 / 7 / 32 / 128 rows — ties to the lowest
    index across slices, all -inf rows to 0 — mixes with sampled rows (handled whole by one workgroup), and
    re-arms its tickets (repeated calls, as under graph replay)."""
    v = 128256
    part = torch.zeros(128 * 32, dtype=torch.int32, device=dev)
    cnt = torch.zeros(128, dtype=torch.int32, device=dev)
    for rows in (1, 7, 32, 128):
        lg = (torch.randn(rows, v, device=dev) * 3).to(torch.bfloat16)
        lg[0, 5] = lg[0, v - 3] = 100.0           # a tie in the first and last slices: the first wins
        if rows > 1:
            lg[1] = float("-inf")
        for _ in range(3):
            got = ops.sample(lg, scratch=(part, cnt)).cpu()
            want = lg.float().argmax(-1).cpu()
            if rows > 1:
                want[1] = 0
            assert torch.equal(got, want), (rows, got[:8], want[:8])
        assert int(cnt.abs().sum()) == 0
    lg = (torch.randn(32, v, device=dev) * 3).to(torch.bfloat16)
    temp = torch.where(torch.arange(32, device=dev) % 2 == 0, 0.0, 0.7).float()
    seeds = torch.arange(32, device=dev, dtype=torch.long)
    steps = torch.zeros(32, device=dev, dtype=torch.long)
    a = ops.sample(lg, temp, None, None, seeds, steps, scratch=(part, cnt)).cpu()
    b = ops.sample(lg, temp, None, None, seeds, steps).cpu()   # one workgroup per row
    assert torch.equal(a, b)
    assert torch.equal(a[::2], lg.float().argmax(-1).cpu()[::2])


def test_sampling_distribution(dev):
    v = 1024
    probs = torch.zeros(v)
    probs[:4] = torch.tensor([0.4, 0.3, 0.2, 0.1])
    logits = torch.log(probs.clamp_min(1e-30)).to(torch.bfloat16)
    n = 4000
    rows = logits[None].repeat(n, 1).to(dev)
    temp = torch.ones(n, device=dev)
    seeds = torch.arange(n, device=dev, dtype=torch.long) * 7919
    steps = torch.zeros(n, device=dev, dtype=torch.long)
    s = ops.sample(rows, temp, None, None, seeds, steps).cpu()
    freq = torch.bincount(s, minlength=v)[:4].float() / n
    assert (freq - probs[:4]).abs().max() < 0.03, freq


def test_block_movers(dev):
    pool = torch.randn(6, 10, 2, 16, 128, device=dev, dtype=torch.bfloat16)
    ref_pool = pool.clone()
    pairs = torch.tensor([[1, 7], [3, 8]], device=dev)
    ops.copy_blocks(pool, pairs)
    ref_pool[:, 7] = ref_pool[:, 1]
    ref_pool[:, 8] = ref_pool[:, 3]
    assert torch.equal(pool, ref_pool)
    ids = torch.tensor([2, 5, 9], device=dev)
    buf = ops.gather_blocks(pool, ids)
    assert torch.equal(buf.view(3, 6, -1)[1], pool[:, 5].reshape(6, -1))
    other = torch.zeros_like(pool)
    ops.scatter_blocks(other, ids, buf)
    assert torch.equal(other[:, ids], pool[:, ids])


@pytest.mark.parametrize("t", [5, 32, 77, 200, 600])  # decode streaming (<= 128) / grouped kernel / hipBLASLt
def test_moe(dev, t):
    h, inter, e, k = 512, 256, 8, 2
    x = torch.randn(t, h, device=dev, dtype=torch.bfloat16)
    gating = torch.randn(t, e, device=dev, dtype=torch.bfloat16)
    w13 = torch.randn(e, 2 * inter, h, device=dev, dtype=torch.bfloat16) / math.sqrt(h)
    w2 = torch.randn(e, h, inter, device=dev, dtype=torch.bfloat16) / math.sqrt(inter)
    w, ids = ops.topk_softmax(gating, k)
    wr, idr = ref.topk_softmax(gating, k)
    # bf16 router logits can tie: compare the selected sets and the weights in sorted order
    assert torch.equal(ids.sort(-1).values.cpu(), idr.sort(-1).values.cpu())
    close(w.sort(-1).values, wr.sort(-1).values, atol=1e-4)
    close(ops.moe_forward(x, w13, w2, gating, k), ref.moe_forward(x, w13, w2, gating, k), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("t,h,e,k", [(32, 4096, 8, 2), (48, 1024, 16, 4), (300, 512, 8, 2)])
def test_moe_route_fused(dev, t, h, e, k):
    """Fused decode routing (router GEMV + softmax + top-k in one launch; t = 300 takes the GEMM path)
    against fp32 logits rounded to bf16 -> reference top-k softmax. Rows whose k-th and (k+1)-th
    logits tie within bf16 rounding may legitimately pick either expert: there only the weights of
    the shared picks are compared."""
    x = torch.randn(t, h, device=dev, dtype=torch.bfloat16)
    wg = torch.randn(e, h, device=dev, dtype=torch.bfloat16) / math.sqrt(h)
    w, ids = ops.moe_route(x, wg, k)
    logits = (x.float() @ wg.float().t()).to(torch.bfloat16).cpu()
    wr, idr = ref.topk_softmax(logits, k)
    srt = logits.float().sort(-1, descending=True).values
    clear = (srt[:, k - 1] - srt[:, k]) > 2e-2 * srt[:, k - 1].abs().clamp(min=1.0)
    got = ids.cpu().long()
    assert torch.equal(got[clear].sort(-1).values, idr.long()[clear].sort(-1).values)
    assert clear.float().mean() > 0.6  # near-ties are rare: most rows must be checked
    close(w.cpu()[clear], wr[clear], atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("t", [8, 32, 48, 100, 128])
@pytest.mark.parametrize("skew", [True, False])
def test_moe_decode_grouped(dev, t, skew):
    """Grouped decode GEMM: 16-row activation image when all experts together have <= 16 rows (t = 8,
    top-2), 32 / 64 / 128-row images above (the step's row bucket bounds any expert's group); skew routes
    every token to experts 0 and 1 (t rows each, six idle experts that must read nothing and write
    nothing)."""
    h, inter, e, k = 1024, 512, 8, 2
    x = torch.randn(t, h, device=dev, dtype=torch.bfloat16)
    w13 = torch.randn(e, 2 * inter, h, device=dev, dtype=torch.bfloat16) / math.sqrt(h)
    w2 = torch.randn(e, h, inter, device=dev, dtype=torch.bfloat16) / math.sqrt(inter)
    if skew:
        ids = torch.tensor([[0, 1]] * t, device=dev, dtype=torch.int32)
    else:
        ids = torch.stack([torch.randperm(e, device=dev)[:k] for _ in range(t)]).to(torch.int32)
    w = torch.softmax(torch.randn(t, k, device=dev), -1)
    want = ref.moe_experts(x, w13, w2, w, ids)
    close(ops.moe_apply(x, w13, w2, w, ids, e), want, atol=3e-2, rtol=3e-2)
    # decode epilogue form: residual += output, row statistics of the new residual (one launch)
    h0 = torch.randn(t, h, device=dev, dtype=torch.bfloat16)
    hres, ssp = h0.clone(), torch.zeros(1, ops.SSP_LD, device=dev)
    ops.moe_apply(x, w13, w2, w, ids, e, residual=hres, ssp=ssp)
    close(hres, h0.float() + want.float(), atol=5e-2, rtol=3e-2)
    close(ssp[0, :t], hres.float().pow(2).sum(-1), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("m,n,k", [(1, 4096, 4096), (7, 6144, 4096), (32, 4096, 14336), (32, 1024, 256),
                                   (16, 4096, 4096), (17, 6144, 4096),
                                   (20, 128256, 4096)])
def test_gemm_decode(dev, m, n, k):
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    y = ops.linear(x, w)
    r = (x.float() @ w.float().t())
    close(y, r, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("m,inter,k", [(32, 14336, 4096), (5, 2048, 1024)])
def test_gemm_decode_silu(dev, m, inter, k):
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2 * inter, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    y = ops.linear_silu_mul(x, w)
    h = x.float() @ w.float().t()
    r = torch.nn.functional.silu(h[:, :inter]) * h[:, inter:]
    close(y, r, atol=2e-2, rtol=2e-2)


def test_gemm_decode_strided_input(dev):
    big = torch.randn(16, 6144, device=dev, dtype=torch.bfloat16)
    x = big[:, :4096]
    w = torch.randn(512, 4096, device=dev, dtype=torch.bfloat16) / 64
    close(ops.linear(x, w), x.float() @ w.float().t(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("wr,sk", [(32, 1), (64, 4), (64, 2)])
def test_gemm_decode_slab_and_consumers(dev, wr, sk):
    m, h = 11, 4096
    x = torch.randn(m, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.randn(h, 4096, device=dev, dtype=torch.bfloat16) / 64
    slab = ops.linear_slab(x, w, sk, wr)
    assert slab.shape == (sk, m, h)
    close(slab.sum(0), x.float() @ w.float().t(), atol=1e-2, rtol=1e-2)
    res = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    g = torch.randn(h, device=dev, dtype=torch.bfloat16)
    y_ref, r_ref = ref.fused_add_rms_norm(slab.sum(0).to(torch.bfloat16), res.clone(), g, 1e-5)
    r2 = res.clone()
    y = ops.fused_add_rms_norm_slab(slab, r2, g, 1e-5)
    close(r2, r_ref, atol=2e-2, rtol=1e-2)
    close(y, y_ref, atol=5e-2, rtol=3e-2)


def test_rope_and_cache_slab(dev):
    hq, hkv, t, sk, bs, nb = 32, 8, 13, 2, 16, 8
    width = (hq + 2 * hkv) * 128
    slab = torch.randn(sk, t, width, device=dev)
    pos = torch.randint(0, 2000, (t,), device=dev)
    slots = torch.randperm(nb * bs, device=dev)[:t]
    cs = ref.rope_cos_sin(4096, 128, 500000.0, dev)
    kc, vc = _paged(nb, hkv, bs, dev)
    kr, vr = _paged(nb, hkv, bs, dev)
    q = ops.rope_and_cache_slab(slab, pos, cs, slots, kc, vc, hq, hkv, 128)
    qkv = slab.sum(0).to(torch.bfloat16)
    ref.rope_and_cache(qkv, pos.cpu(), cs, slots.cpu(), kr, vr, hq, hkv, 128)
    close(q, qkv[:, : hq * 128], atol=3e-2, rtol=2e-2)
    close(kc, kr, atol=3e-2, rtol=2e-2)
    close(vc, vr, atol=2e-2, rtol=1e-2)


# ---------------------------------------------------------------- fused decode path pieces
@pytest.mark.parametrize("wr,sk,k,m,kc", [(64, 4, 4096, 27, None), (64, 4, 14336, 27, None), (32, 1, 2048, 27, None),
                                          (128, 2, 4096, 27, None), (64, 8, 4096, 27, None), (32, 3, 3072, 27, None),
                                          (64, 4, 4096, 100, 128), (128, 8, 4096, 128, 32), (64, 2, 14336, 64, 256),
                                          (128, 4, 4096, 77, 64), (64, 3, 4096, 27, 256), (32, 5, 8192, 32, 256),
                                          (128, 4, 28672, 32, 128)])  # Llama-3-70B TP=1 down's tile, its K
def test_gemm_decode_residual_mode(dev, wr, sk, k, m, kc):
    """mode 3: resid += x @ w^T with the split-K reduced by the last-arriving workgroup, which
    also writes the per-tile row sums of squares of the new residual."""
    h = 4096
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(h, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    res = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    t = h // wr
    ssp = torch.full((t, ops.SSP_LD), -1.0, device=dev)
    cnt = torch.zeros(t, dtype=torch.int32, device=dev)
    for it in range(2):  # tickets are re-armed: a second launch works too
        r0 = res.clone()
        ops.linear_slab_residual(x, w, res, ssp, cnt, wr, sk, kc=kc)
        expect = (r0.float() + x.float() @ w.float().t()).to(torch.bfloat16)
        close(res, expect, atol=3e-2, rtol=1e-2)
        ss_ref = res.float().pow(2).view(m, t, wr).sum(-1).t()       # [t, m]
        close(ssp[:, :m], ss_ref, atol=1e-2, rtol=1e-3)
        rr = 32 if m <= 32 else (64 if m <= 64 else 128)  # rows of the activation image: padded rows -> 0
        assert torch.all(ssp[:, m:rr] == 0)
        assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("n,k,wr,kc,sk,m", [(1280, 8192, 32, 256, 5, 32), (1280, 8192, 32, 128, 6, 7),
                                            (6144, 4096, 48, 256, 3, 19)])
def test_gemm_decode_uneven_split_slabs(dev, n, k, wr, kc, sk, m):
    """Split-K counts that do not divide K's slots (splits differ by one K-slot): the fp32 slabs sum to x @ w^T,
    row-major and tile-order weights alike."""
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    ref32 = x.float() @ w.float().t()
    a = ops.gemm_decode(x, w, mode=2, wr=wr, sk=sk, kc=kc)
    b = ops.gemm_decode(x, ops.gd_pack_weights(w, wr, kc=kc), mode=2 | 32, wr=wr, sk=sk, kc=kc)
    assert a.shape == (sk, m, n) and torch.equal(a, b)
    close(a.sum(0), ref32, atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("sk", [4, 3])
def test_gemm_decode_residual_mode_is_deterministic(dev, sk):
    """The split-K last arriver sums the slices in slice order whichever slice arrived last: repeated launches
    from the same residual are bit-identical (compile-time and runtime split counts). (Summed in arrival order
    they differed in the last bit of a few elements per launch: profiles/r5_down_qkv_pair_negative.jsonl.)"""
    m, h, k = 19, 4096, 3072 * 4 if sk == 4 else 3072
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(h, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    res0 = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    ssp = torch.zeros(h // 64, ops.SSP_LD, device=dev)
    cnt = torch.zeros(h // 64, dtype=torch.int32, device=dev)
    outs = []
    for _ in range(8):
        r = res0.clone()
        ops.linear_slab_residual(x, w, r, ssp, cnt, 64, sk)
        outs.append((r, ssp.clone()))
    for r, s in outs[1:]:
        assert torch.equal(r, outs[0][0]) and torch.equal(s, outs[0][1])


@pytest.mark.parametrize("m,inter,k,wr,t", [(32, 14336, 4096, 112, 64), (7, 2048, 1024, 64, 64),
                                           (100, 14336, 4096, 112, 64), (64, 2048, 1024, 64, 64),
                                           (32, 3584, 8192, 64, 256), (19, 3584, 8192, 64, 200),
                                           (32, 28672, 8192, 112, 128)])  # Llama-3-70B TP=1 gate/up tile and shape
def test_gemm_decode_rownorm_silu(dev, m, inter, k, wr, t):
    """mode 4: RMSNorm (weight folded into W) as a per-row scale + gate/up + SiLU*mul; the statistics arrive as
    t per-tile partial sums (up to 256 tiles at <= 32 rows: a residual written by wr = 32 tiles of 8,192)."""
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16) * 3
    w = torch.randn(2 * inter, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    ss = x.float().pow(2)
    if k % t:
        t = 1
    ssp = torch.zeros(t, ops.SSP_LD, device=dev)
    ssp[:, :m] = ss.view(m, t, -1).sum(-1).t()
    y = ops.linear_silu_mul_rownorm(x, w, ssp, 1e-5, wr)
    xn = x.float() * torch.rsqrt(ss.mean(-1, keepdim=True) + 1e-5)
    hh = xn @ w.float().t()
    r = torch.nn.functional.silu(hh[:, :inter]) * hh[:, inter:]
    close(y, r, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("mode,n,k,wr,sk", [(0, 1024, 4096, 64, 1), (1, 1792, 4096, 112, 1), (2, 4096, 4096, 64, 4),
                                            (2, 6144, 4096, 48, 2), (4, 2304, 1024, 96, 1)])
def test_gemm_decode_tiled_weights(dev, mode, n, k, wr, sk):
    """Weights pre-packed in the kernel's tile order (ops.gd_pack_weights; one linear 1-KiB read per
    LDS-DMA piece) give bit-identical results to the row-major layout in every epilogue."""
    m = 19
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    rows = 2 * n if mode in (1, 4) else n
    w = torch.randn(rows, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    wt = ops.gd_pack_weights(w, wr, silu=mode in (1, 4))
    if mode == 4:
        ssp = x.float().pow(2).sum(-1).view(1, m)
        ssp_in = torch.zeros(1, ops.SSP_LD, device=dev)
        ssp_in[0, :m] = ssp
        a = ops.linear_silu_mul_rownorm(x, w, ssp_in, 1e-5, wr)
        b = ops.linear_silu_mul_rownorm(x, wt, ssp_in, 1e-5, wr, tiled=True)
    else:
        a = ops.gemm_decode(x, w, mode=mode, wr=wr, sk=sk)
        b = ops.gemm_decode(x, wt, mode=mode | 32, wr=wr, sk=sk)
    assert torch.equal(a, b)
    if mode == 0:
        close(a, x.float() @ w.float().t(), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("g,hkv,big,tiles,sk", [(4, 8, False, 4, 2), (8, 1, False, 4, 2), (1, 4, False, 4, 2),
                                                (4, 8, True, 4, 2), (8, 1, False, 256, 2), (4, 8, True, 130, 2),
                                                (8, 1, "tp8", 128, 4), (8, 1, "tp8", 256, 2)])
def test_attn_decode_fused(dev, g, hkv, big, tiles, sk):
    """Fused prologue: norm scale + qkv slab sum + RoPE at ctx-1 + KV write, then attention.
    big: 32 sequences x 8 kv heads. "tp8": a Llama-3-70B TP=8 shard (32 sequences x 1 kv head, max context
    2,048: two-chunk parts, up to 16 parts merged per pair; parts without the new token stage only the q rows
    of the slabs). tiles: norm-statistics tiles (up to 256). sk: qkv split-K slabs."""
    hq, bs, d = hkv * g, 16, 128
    hid = 1024
    ctxs = [1, 17, 200, 777, 2049]
    max_ctx = 4096
    if big == "tp8":
        ctxs = [1, 17, 64, 65, 129, 200, 1024, 1025, 2048] + [400 + 29 * i for i in range(23)]
        max_ctx = 2048
    elif big:
        ctxs = [1, 17, 64, 65, 129, 200, 777, 2049] + [400 + 29 * i for i in range(24)]
    n = len(ctxs)
    width = (hq + 2 * hkv) * d
    _, kc, vc, bt, _, ctx, _ = _make_seqs([1] * n, ctxs, hkv, bs, dev, g)
    bt_wide = torch.zeros(n, max(max_ctx // bs, bt.shape[1]), dtype=torch.int32, device=dev)
    bt_wide[:, : bt.shape[1]] = bt
    slab = torch.randn(sk, n, width, device=dev) * 0.7   # normalised q/k/v ~ N(0, 1): realistic scores
    ssv = (torch.rand(n, device=dev) + 0.5) * hid
    ssp = torch.zeros(tiles, ops.SSP_LD, device=dev)
    ssp[:, :n] = (ssv / tiles)[None, :]                 # `tiles` tiles summing to ssv
    slots = torch.tensor([int(bt[i, (c - 1) // bs]) * bs + (c - 1) % bs for i, c in enumerate(ctxs)],
                         dtype=torch.long, device=dev)
    slots[1] = -1                                        # a padded row: no cache write
    pos = (ctx - 1).long()
    cs = ref.rope_cos_sin(8192, d, 500000.0, dev)
    maxp = ops.decode_partials(max_ctx)
    po = torch.empty(n * hq * maxp * d, device=dev)
    pm = torch.empty(n * hq * maxp * 2, device=dev)
    cnt = torch.zeros(n * hkv, dtype=torch.int32, device=dev)
    kr, vr = kc.clone(), vc.clone()
    scale = 1 / math.sqrt(d)
    out = ops.attn_decode_fused(slab, ssp, pos, cs, slots, kc, vc, bt_wide, ctx, max_ctx, hq, hkv, scale, 1e-5,
                                hid, po, pm, cnt)
    # reference: normalise the summed projection, rope + cache, attention
    rn = torch.rsqrt(ssv / hid + 1e-5)
    qkv = (slab.sum(0) * rn[:, None]).to(torch.bfloat16)
    slots_ref = slots.clone()
    ref.rope_and_cache(qkv, pos.cpu(), cs, slots_ref.cpu(), kr, vr, hq, hkv, d)
    # row 1 is "padded": its new token is not written; the kernel still attends to it via LDS
    blk, off = int(bt[1, (ctxs[1] - 1) // bs]), (ctxs[1] - 1) % bs
    k1 = ref.apply_rope(qkv[1:2, hq * d:(hq + hkv) * d].view(1, hkv, d), pos[1:2].cpu(), cs)
    kr2, vr2 = kr.clone(), vr.clone()
    kr2[blk, :, off] = k1[0]
    vr2[blk, :, off] = qkv[1, (hq + hkv) * d:].view(hkv, d)
    cu = torch.arange(n + 1, dtype=torch.int32, device=dev)
    r = ref.attention(qkv[:, : hq * d], kr2, vr2, bt, cu, ctx, hq, hkv, scale).reshape(n, -1)
    close(out, r, atol=3e-2, rtol=3e-2)
    # the cache got the new tokens (except the padded row); the kernel rotates before rounding
    close(kc, kr, atol=3e-2, rtol=2e-2)
    close(vc, vr, atol=3e-2, rtol=2e-2)
    assert int(cnt.abs().sum()) == 0


def test_residual_add_sumsq(dev):
    m, h = 13, 8192
    res = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    x = torch.randn(m, h, device=dev, dtype=torch.bfloat16)
    expect = (res.float() + x.float()).to(torch.bfloat16)
    ssp = torch.full((1, 32), -1.0, device=dev)
    ops.residual_add_sumsq(res, x, ssp)
    assert torch.equal(res, expect)
    close(ssp[0, :m], expect.float().pow(2).sum(-1), atol=1e-2, rtol=1e-4)


# ------------------------------------------------------- decode GEMM at M <= 128
@pytest.mark.parametrize("m", [33, 64, 100, 128])
@pytest.mark.parametrize("wr,kc", [(64, 256), (112, 128), (64, 128), (128, 64), (128, 32), (64, 32)])
def test_gemm_decode_large_m(dev, m, wr, kc):
    """Every tile at batch sizes past 32 rows (64- and 128-row activation images, waves split the rows),
    plain and silu epilogues, against fp32; tiles without a 64/128-row image must refuse loudly."""
    k, n = 4096, 1792
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2 * n, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    try:
        y = ops.gemm_decode(x, w[:n], 0, wr, 1, kc=kc)
    except RuntimeError as e:  # (wr, kc) has no image for this many rows: a clean launch error
        assert "invalid" in str(e).lower() or "unsupported" in str(e).lower(), e
        return
    close(y, x.float() @ w[:n].float().t(), atol=2e-2, rtol=2e-2)
    if wr in (64, 128) or (wr == 112 and n % 56 == 0):
        ys = ops.gemm_decode(x, w, 1, wr, 1, kc=kc)
        h = x.float() @ w.float().t()
        close(ys, torch.nn.functional.silu(h[:, :n]) * h[:, n:], atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m,wr,kc,sk", [(64, 128, 32, 4), (128, 128, 64, 2), (100, 64, 128, 2), (48, 128, 32, 8)])
def test_gemm_decode_large_m_slabs_and_tiled(dev, m, wr, kc, sk):
    """Split-K slabs and tile-order packed weights with the small K slots (swizzle of 128- and 64-byte rows)."""
    k, n = 4096, 2048
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) / math.sqrt(k)
    a = ops.gemm_decode(x, w, 2, wr, sk, kc=kc)
    close(a.sum(0), x.float() @ w.float().t(), atol=2e-2, rtol=2e-2)
    wt = ops.gd_pack_weights(w, wr, kc=kc)
    b = ops.gemm_decode(x, wt, 2 | 32, wr, sk, kc=kc)
    assert torch.equal(a, b)


@pytest.mark.parametrize("rows", [1, 7, 32, 128])
def test_embed_sumsq_matches_gather_and_fp32_sumsq(dev, rows):
    """The decode step's fused embedding gather + first-norm statistics (norm_act.hip embed_sumsq) against
    torch's gather and an fp32 sum of squares of the gathered bf16 rows; the statistics row is [1, 128]."""
    table = (torch.randn(5000, 4096, device=dev) * 0.05).to(torch.bfloat16)
    ids = torch.randint(0, 5000, (rows,), device=dev)
    ssp = torch.full((1, ops.SSP_LD), -1.0, device=dev)
    h, s = ops.embed_sumsq(ids, table, ssp)
    assert s is ssp
    want = torch.nn.functional.embedding(ids, table)
    assert torch.equal(h, want)
    ref = want.float().pow(2).sum(-1)
    torch.testing.assert_close(ssp[0, :rows], ref, rtol=1e-5, atol=1e-5)
    assert torch.all(ssp[0, rows:] == -1.0)  # rows past M untouched


@pytest.mark.parametrize("n,k,wr,kc,sk,m", [(3584, 8192, 64, 256, 2, 32), (3584, 8192, 64, 256, 2, 7),
                                           (2048, 1024, 64, 128, 4, 32), (2048, 1024, 128, 64, 2, 1),
                                           # the 70B TP=8 shard's 64- / 128-row tiles (DECODE_SILU_SPLITK_CFG)
                                           (3584, 8192, 112, 128, 4, 64), (3584, 8192, 112, 128, 4, 50),
                                           (3584, 8192, 64, 128, 2, 128), (3584, 8192, 64, 128, 2, 100)])
def test_gate_up_split_k_silu_matches_full_k(dev, n, k, wr, kc, sk, m):
    """Mode 6 (the norm-scaled SiLU gate/up with K split over sk workgroups, fp32 partial slabs, last-arriver
    finish) against mode 4 (one pass) and an fp32 reference; the tickets are re-armed for the next launch."""
    w = (torch.randn(2 * n, k, device=dev) * 0.02).to(torch.bfloat16)
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    ssp = (torch.rand(3, ops.SSP_LD, device=dev) * k * 0.1).float()
    wt = ops.gd_pack_weights(w, wr, silu=True, kc=kc)
    slab = torch.empty(sk * m * 2 * n, dtype=torch.float32, device=dev)
    cnt = torch.zeros(n // (wr // 2), dtype=torch.int32, device=dev)
    got = ops.linear_silu_mul_rownorm(x, wt, ssp, 1e-5, wr, tiled=True, kc=kc, sk=sk, slab=slab, counters=cnt)
    again = ops.linear_silu_mul_rownorm(x, wt, ssp, 1e-5, wr, tiled=True, kc=kc, sk=sk, slab=slab, counters=cnt)
    one = ops.linear_silu_mul_rownorm(x, wt, ssp, 1e-5, wr, tiled=True, kc=kc)
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0
    assert torch.equal(got, again)  # deterministic (slices summed in slice order)
    r = torch.rsqrt(ssp[:, :m].sum(0) / k + 1e-5)[:, None]
    y = (x.float() @ w.float().t()) * r
    ref = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    for out in (got, one):
        err = float((out.float() - ref).norm() / ref.norm())
        assert err < 1e-2, err
    assert float((got.float() - one.float()).norm() / one.float().norm()) < 5e-3


def test_prefill_gemm_table_loads_and_matches_fp32(dev):
    """The prefill GEMM table (src/ops/gemm_table.py) loads read-only on this stack (TunableOp on, tuning off)
    and a listed shape (Llama-3-8B qkv at 2,048 tokens) still matches the fp32 product."""
    from src.ops.gemm_table import enable_prefill_gemm_table, table_entries

    import torch.cuda.tunable as tun

    assert enable_prefill_gemm_table(), "table rejected by this PyTorch / ROCm stack"
    assert tun.is_enabled() and not tun.tuning_is_enabled()
    assert (6144, 2048, 4096) in table_entries()
    x = torch.randn(2048, 4096, device=dev).to(torch.bfloat16)
    w = (torch.randn(6144, 4096, device=dev) * 0.02).to(torch.bfloat16)
    y = torch.nn.functional.linear(x, w)
    close(y, x.float() @ w.float().t(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("m", [1, 7, 32, 128])
@pytest.mark.parametrize("n,wr,kc", [(128256, 128, 128), (32000, 64, 128)])
def test_lm_head_argmax_candidates(dev, m, n, wr, kc):
    """The decode LM head with per-column-tile greedy candidates (ops.linear_tiled_argmax): the same logits bit
    for bit as the plain tiled GEMM, and the candidates reduce (ops.sample(lm_part=...)) to torch.argmax of those
    logits — lowest index on a tie (rows 100 and n - 900 are made identical and dominant for every token);
    sampled rows (temperature > 0) ignore the candidates and draw exactly as without them."""
    k = 4096
    g = torch.Generator(device=dev).manual_seed(m + n)
    x = torch.randn(m, k, device=dev, generator=g).abs().to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    w[100] = 0.05
    w[n - 900] = 0.05
    wt = ops.gd_pack_weights(w, wr, kc=kc)
    parts = torch.zeros(m, n // wr, 2, dtype=torch.int32, device=dev)
    y = ops.linear_tiled_argmax(x, wt, wr, kc, parts)
    assert torch.equal(y, ops.linear_tiled(x, wt, wr, kc))
    want = torch.argmax(y.float(), dim=-1)
    assert bool((want == 100).all())
    got = ops.sample(y, lm_part=parts)
    assert torch.equal(got, want)
    # without the tie: the plain argmax of random logits, and candidates = per-tile maxima
    w[100] = w[101]
    w[n - 900] = w[n - 901]
    wt = ops.gd_pack_weights(w, wr, kc=kc)
    y = ops.linear_tiled_argmax(x, wt, wr, kc, parts)
    assert torch.equal(ops.sample(y, lm_part=parts), torch.argmax(y.float(), dim=-1))
    tiles = y.float().view(m, n // wr, wr)
    assert torch.equal(parts[..., 0].view(torch.float32), tiles.max(-1).values)
    assert torch.equal(parts[..., 1].long(), tiles.argmax(-1) + torch.arange(0, n, wr, device=dev))
    temp = torch.full((m,), 0.8, device=dev)
    seeds = torch.arange(m, device=dev, dtype=torch.long)
    steps = torch.zeros(m, device=dev, dtype=torch.long)
    assert torch.equal(ops.sample(y, temp, seeds=seeds, steps=steps, lm_part=parts),
                       ops.sample(y, temp, seeds=seeds, steps=steps))


@pytest.mark.parametrize("rows,n_real", [(32, 32), (32, 29), (8, 8)])
def test_sample_advance_matches_sample_then_advance(dev, rows, n_real):
    """ops.sample_advance (sampling from the LM head's candidates + the decode step's input advance in one launch)
    leaves every buffer exactly as ops.sample(lm_part=...) followed by ops.decode_advance: tokens, ids, positions,
    context lengths, slots, steps, the window's token row and step counter — with greedy and sampled rows, padded
    rows past n_real, and the row ticket re-armed for the next launch (two steps in a row)."""
    n, wr, kc, k, bs, width, kmax = 32000, 64, 128, 4096, 16, 8, 8
    g = torch.Generator(device=dev).manual_seed(rows + n_real)
    x = torch.randn(rows, k, device=dev, generator=g).to(torch.bfloat16)
    wt = ops.gd_pack_weights((torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16), wr, kc=kc)
    parts = torch.zeros(rows, n // wr, 2, dtype=torch.int32, device=dev)
    logits = ops.linear_tiled_argmax(x, wt, wr, kc, parts)
    temp = torch.zeros(rows, device=dev)
    temp[1::3] = 0.7  # some sampled rows
    topk = torch.zeros(rows, dtype=torch.int32, device=dev)
    topp = torch.ones(rows, device=dev)
    seeds = torch.arange(rows, dtype=torch.long, device=dev) + 11

    def state():
        pos = torch.randint(0, width * bs - 2, (rows,), device=dev, generator=g)
        return {"ids": torch.zeros(rows, dtype=torch.long, device=dev), "pos": pos,
                "ctx": (pos + 1).to(torch.int32), "slots": torch.zeros(rows, dtype=torch.long, device=dev),
                "bt": torch.randint(0, 1000, (rows, width), dtype=torch.int32, device=dev, generator=g),
                "step": torch.randint(0, 50, (rows,), device=dev, generator=g),
                "tokens": torch.full((2 * kmax, rows), -1, dtype=torch.long, device=dev),
                "ctl": torch.tensor([3, n_real], dtype=torch.int32, device=dev),
                "out": torch.zeros(rows, dtype=torch.long, device=dev)}

    a = state()
    b = {kk: v.clone() for kk, v in a.items()}
    ticket = torch.zeros(1, dtype=torch.int32, device=dev)
    table = torch.randn(n, 512, device=dev, generator=g).to(torch.bfloat16)
    h_out = torch.zeros(rows, 512, dtype=torch.bfloat16, device=dev)
    ssp_out = torch.zeros(1, ops.SSP_LD, device=dev)
    for _ in range(2):
        ops.sample(logits, temp, topk, topp, seeds, a["step"], out=a["out"], lm_part=parts)
        ops.decode_advance(a["out"], a["ids"], a["pos"], a["ctx"], a["slots"], a["bt"], a["step"], a["tokens"],
                           a["ctl"][0:1], a["ctl"][1:2], rows, bs)
        ops.sample_advance(logits, temp, topk, topp, seeds, b["step"], b["out"], parts, b["ids"], b["pos"], b["ctx"],
                           b["slots"], b["bt"], b["tokens"], b["ctl"][0:1], b["ctl"][1:2], bs, ticket,
                           embed=(table, h_out, ssp_out.view(-1)))
    torch.cuda.synchronize()
    for kk in a:
        assert torch.equal(a[kk], b[kk]), kk
    assert int(ticket.item()) == 0 and int(b["ctl"][0].item()) == 5
    # the next step's embedding rows and statistics: bit-identical to embed_sumsq of the advanced ids
    ssp_ref = torch.zeros(1, ops.SSP_LD, device=dev)
    h_ref, _ = ops.embed_sumsq(a["ids"][:rows], table, ssp_ref)
    assert torch.equal(h_out, h_ref) and torch.equal(ssp_out[0, :rows], ssp_ref[0, :rows])


@pytest.mark.parametrize("wr", [48, 96, 112])
def test_lm_head_argmax_refuses_non_power_of_two_lanes(dev, wr):
    """The candidate epilogue merges a row's wr / 8 lanes with xor shuffles: tiles whose lane count is not a power
    of two (wr = 48 / 96 / 112) would mix rows, so the launcher refuses them instead of writing wrong candidates
    (ADVICE r5)."""
    m, n, k = 4, wr * 8, 512
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
    wt = ops.gd_pack_weights(w, wr, kc=128)
    parts = torch.zeros(m, n // wr, 2, dtype=torch.int32, device=dev)
    with pytest.raises(RuntimeError):
        ops.linear_tiled_argmax(x, wt, wr, 128, parts)
    torch.cuda.synchronize()


@pytest.mark.parametrize("n,k,wr,kc,sk,rows", [(8192, 1024, 32, 128, 1, 32), (8192, 3584, 32, 256, 1, 32),
                                               (8192, 3584, 32, 256, 1, 7), (4096, 2048, 32, 128, 2, 32)])
def test_half_ring_residual_gemm_matches_full_ring(dev, n, k, wr, kc, sk, rows):
    """The half-LDS ring of the residual-updating decode GEMM (mode 3, two workgroups per CU: the TP exchange's
    residency form at the 70B TP=8 shard's o / down shapes) gives bit-identical residual and statistics to the full
    ring, and its occupancy is what the residency rule assumes (2 per CU vs 1)."""
    assert ops.gd_occupancy(3, wr, kc, sk, 32, False) == 1
    assert ops.gd_occupancy(3, wr, kc, sk, 32, True) >= 2
    g = torch.Generator(device=dev).manual_seed(n + k + rows)
    x = (torch.randn(rows, k, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    wt = ops.gd_pack_weights(w, wr, kc=kc)
    r0 = torch.randn(rows, n, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for half in (False, True):
        r = r0.clone()
        ssp = torch.zeros(n // wr, ops.SSP_LD, device=dev)
        cnt = torch.zeros(n // wr, dtype=torch.int32, device=dev)
        ops.linear_slab_residual(x, wt, r, ssp, cnt, wr, sk, tiled=True, kc=kc, half_ring=half)
        outs.append((r, ssp))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    want = r0.float() + x.float() @ w.float().t()
    assert float((outs[1][0].float() - want).abs().max()) < 0.1


def test_tp8_shard_plan_takes_the_half_ring_on_real_occupancy():
    """at the 70B TP=8 tile counts (N = 8,192, wr = 32, grid = 256) the fused exchange is taken only
    under the residency rule evaluated on the real occupancy of the exact instantiation (hipOccupancy...): one
    workgroup per CU with the full LDS ring fails it, so the plan takes the half-LDS ring (two per CU)."""
    from src.models.llama import CausalLM
    from src.models.presets import get_preset
    from src.parallel.custom_allreduce import fused_exchange_ok
    from src.parallel.tp import TPContext

    cus = torch.cuda.get_device_properties(0).multi_processor_count

    class NodeTP(TPContext):  # one rank per GPU, the IPC path assumed up
        def fused_row_parallel(self, n_tiles, grid=0, per_cu=0):
            return fused_exchange_ok(n_tiles, grid, per_cu, 1, cus)

    m = object.__new__(CausalLM)
    m.arch = get_preset("llama3-70b")
    m.tp = NodeTP(rank=0, world_size=8)
    m.hq, m.hkv, m.head_dim, m.inter = 8, 1, 128, 28672 // 8
    m.layers = [type("L", (), {"qkv": torch.empty(1280, 8192, device="meta")})()]
    assert ops.gd_occupancy(3, 32, 128, 1, 32, False) == 1 and ops.gd_occupancy(3, 32, 256, 1, 32, False) == 1
    p = m.decode_plan(32)
    assert p["tp_fused"] and p["o"][0] == 32 and p["down"][0] == 32 and p["o_half"] and p["down_half"], p
