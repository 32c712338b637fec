"""Local HF-format checkpoints (config.json + safetensors): round trip through the loader with
non-trivial RMSNorm weights (folded on load), sharded files, and per-rank TP slicing."""

import os

import pytest
import torch

from src.config import EngineConfig
from src.engine import LLMEngine
from src.models.llama import CausalLM
from src.models.loader import arch_from_hf_config, is_hf_checkpoint, load_checkpoint, save_hf_checkpoint
from src.models.presets import get_preset
from src.parallel.tp import TPContext
from src.preproc import SamplingParams

PROMPTS = [[5, 9, 33, 12, 7] * 5, [100, 200, 300], list(range(3, 60))]


def _cfg():
    return EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, num_kv_blocks=64, max_latency_ms=0.0)


def _model_with_norms(preset, seed=7):
    m = CausalLM(get_preset(preset), "cpu", dtype=torch.float32, seed=seed, max_position=256)
    g = torch.Generator().manual_seed(seed)
    norms = {}
    for i, lw in enumerate(m.layers):   # checkpoint-like norm weights, applied unfolded
        lw.ln1.copy_(torch.rand(lw.ln1.shape, generator=g) + 0.5)
        lw.ln2.copy_(torch.rand(lw.ln2.shape, generator=g) + 0.5)
    m.norm.copy_(torch.rand(m.norm.shape, generator=g) + 0.5)
    return m


@pytest.mark.parametrize("preset,shards", [("llama-tiny", 3), ("mixtral-tiny", 2)])
def test_roundtrip_generates_identically(tmp_path, preset, shards):
    src = _model_with_norms(preset)
    ref = LLMEngine(src, _cfg(), 256)
    ref.eos_token_id = None
    expect = ref.generate(PROMPTS, SamplingParams(max_tokens=6))
    path = str(tmp_path / "ckpt")
    save_hf_checkpoint(src, path, shards=shards)
    assert is_hf_checkpoint(path) and len([f for f in os.listdir(path) if f.endswith(".safetensors")]) == shards
    arch = arch_from_hf_config(path)
    assert (arch.hidden_size, arch.num_layers, arch.num_experts) == (src.arch.hidden_size, src.arch.num_layers,
                                                                       src.arch.num_experts)
    eng = LLMEngine.from_pretrained(path, device="cpu", cfg=_cfg(), max_model_len=256, capture=False,
                                    dtype=torch.float32)
    eng.eos_token_id = None
    if not arch.is_moe:  # dense: norms folded into Wqkv / Wgate_up, norm weights now ones
        assert eng.model.norms_folded and all(bool((lw.ln1 == 1).all()) for lw in eng.model.layers)
    assert eng.generate(PROMPTS, SamplingParams(max_tokens=6)) == expect


def test_tp_slices(tmp_path):
    src = CausalLM(get_preset("llama-tiny"), "cpu", dtype=torch.float32, seed=11, max_position=256)
    path = str(tmp_path / "ckpt")
    save_hf_checkpoint(src, path, shards=2)
    arch = arch_from_hf_config(path)
    ranks = []
    for r in range(2):
        m = CausalLM(arch, "cpu", dtype=torch.float32, tp=TPContext(rank=r, world_size=2), max_position=256)
        load_checkpoint(m, path)
        ranks.append(m)
    d, lw0, lw1, full = src.head_dim, ranks[0].layers[1], ranks[1].layers[1], src.layers[1]
    hq, hkv = ranks[0].hq, ranks[0].hkv
    nq, nkv = src.hq, src.hkv
    q_full = full.qkv[: nq * d]
    assert torch.equal(torch.cat([lw0.qkv[: hq * d], lw1.qkv[: hq * d]]), q_full)
    assert torch.equal(torch.cat([lw0.qkv[hq * d:(hq + hkv) * d], lw1.qkv[hq * d:(hq + hkv) * d]]),
                       full.qkv[nq * d:(nq + nkv) * d])
    assert torch.equal(torch.cat([lw0.o, lw1.o], 1), full.o)
    i = ranks[0].inter
    assert torch.equal(torch.cat([lw0.gate_up[:i], lw1.gate_up[:i]]), full.gate_up[: 2 * i])
    assert torch.equal(torch.cat([lw0.down, lw1.down], 1), full.down)
