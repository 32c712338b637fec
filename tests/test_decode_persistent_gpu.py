"""The persistent decode-step kernel (csrc/kernels/decode_persistent.hip): every layer of a dense decode step
in one launch. Its arithmetic is the multi-launch fused path's (gemm_decode.hip SPLIT-0 tiles at KC 128, the
v3 attention's one-part FUSED path, split-K slabs in slice order), so with the same tiles the two must agree
BIT FOR BIT — the residual stream after the last layer and the new tokens' K / V in the paged cache."""

import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

os.environ["DIE_PERSISTENT"] = "1"

from src import ops  # noqa: E402
from src.models.llama import AttnMetadata, CausalLM  # noqa: E402
from src.models.presets import get_preset  # noqa: E402


def _setup(preset, n_layers, M, ctxs, seed=0, max_ctx=1024):
    dev = torch.device("cuda:0")
    arch = get_preset(preset, num_layers=n_layers)
    m = CausalLM(arch, dev, seed=seed, max_position=max_ctx + 16)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    bs = 16
    nbps = max_ctx // bs
    nblocks = M * nbps + 8
    pool = (torch.randn(n_layers, 2, nblocks, m.hkv, bs, 128, generator=g, device=dev) * 0.7).to(torch.bfloat16)
    perm = torch.randperm(nblocks - 8, generator=torch.Generator().manual_seed(seed + 2))
    bt = perm[: M * nbps].view(M, nbps).to(torch.int32).to(dev)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=dev)
    pos = (ctx - 1).long()
    slots = (bt[torch.arange(M, device=dev), pos // bs].long() * bs + pos % bs)
    ids = torch.randint(0, arch.vocab_size, (M,), generator=g, device=dev)
    maxp = ops.decode_partials(max_ctx)
    meta_kw = dict(part_o=torch.empty(M * m.hq * maxp * 128, dtype=torch.float32, device=dev),
                   part_ml=torch.empty(M * m.hq * maxp * 2, dtype=torch.float32, device=dev),
                   attn_cnt=torch.zeros(M * m.hkv, dtype=torch.int32, device=dev))
    return m, pool, bt, ctx, pos, slots, ids, meta_kw, max_ctx


def _run_both(preset, n_layers, M, ctxs, seed=0):
    m, pool, bt, ctx, pos, slots, ids, meta_kw, max_ctx = _setup(preset, n_layers, M, ctxs, seed)
    sc = m.alloc_decode_scratch(M)
    assert m.prepare_persistent(pool, sc), "no persistent instantiation for this shape"
    cfg = sc["persistent"]["cfg"]
    # the multi-launch fused path on the SAME tiles as the persistent kernel
    plan = {"qkv": (cfg["wrq"], 128, cfg["skq"]), "o": (cfg["wro"], 128, cfg["sko"]),
            "down": (cfg["wrd"], 128, cfg["skd"]), "gate_up": (cfg["wrg"], 128)}
    ref_sc = {k: v for k, v in sc.items() if k != "persistent"}
    ref_sc["plans"] = {b: plan for b in sc["plans"]}
    outs = {}
    for name, scratch in (("multi", ref_sc), ("persistent", sc)):
        p = pool.clone()
        meta = AttnMetadata(False, slots, bt, ctx, max_ctx=max_ctx, scratch=scratch, **meta_kw)
        with torch.inference_mode():
            hid = m.forward(ids, pos, meta, p)
        torch.cuda.synchronize()
        outs[name] = (hid.clone(), p)
    err = int(sc["persistent"]["err"].item())
    return outs, err


@pytest.mark.parametrize("M", [32, 7, 1])
def test_persistent_matches_multi_launch_mini(M):
    """llama-mini (4 layers, 8 q / 2 kv heads): contexts within one 128-key chunk (the multi-launch attention
    then also runs one part per pair)."""
    ctxs = [1 + (37 * i) % 128 for i in range(M)]
    outs, err = _run_both("llama-mini", 4, M, ctxs)
    assert err == 0
    (h0, p0), (h1, p1) = outs["multi"], outs["persistent"]
    assert torch.isfinite(h1.float()).all()
    assert torch.equal(h0, h1), float((h0.float() - h1.float()).abs().max())
    assert torch.equal(p0, p1)


def test_persistent_matches_multi_launch_8b_shapes():
    """Llama-3-8B layer shapes (2 layers), the bench's 32 rows at 500-640 keys: every phase has one task per
    CU, attention spans 4-5 chunks per task; bit-exact against the multi-launch path with the same tiles."""
    ctxs = [500 + 4 * i for i in range(32)]
    outs, err = _run_both("llama3-8b", 2, 32, ctxs, seed=3)
    assert err == 0
    (h0, p0), (h1, p1) = outs["multi"], outs["persistent"]
    assert torch.isfinite(h1.float()).all()
    assert torch.equal(h0, h1), float((h0.float() - h1.float()).abs().max())
    assert torch.equal(p0, p1)


def test_persistent_repeated_launches_are_identical():
    """The counters are re-zeroed and the split-K tickets re-armed by every launch: the same inputs give the
    same bits on every call (also under hipGraph replay)."""
    m, pool, bt, ctx, pos, slots, ids, meta_kw, max_ctx = _setup("llama-mini", 4, 32, [100] * 32, seed=5)
    sc = m.alloc_decode_scratch(32)
    assert m.prepare_persistent(pool, sc)
    meta = AttnMetadata(False, slots, bt, ctx, max_ctx=max_ctx, scratch=sc, **meta_kw)
    res = []
    with torch.inference_mode():
        for _ in range(3):
            res.append(m.forward(ids, pos, meta, pool).clone())
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.forward(ids, pos, meta, pool)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph):
            out = m.forward(ids, pos, meta, pool)
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            res.append(out.clone())
    assert int(sc["persistent"]["err"].item()) == 0
    for r in res[1:]:
        assert torch.equal(r, res[0])
