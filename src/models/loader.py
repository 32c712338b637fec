"""
Local HuggingFace-format checkpoints: ``config.json`` + ``*.safetensors`` (Llama / Llama-3 /
Mistral / Mixtral names). No network: the directory must already be on disk.

* :func:`arch_from_hf_config` maps the HF config onto :class:`ArchConfig`.
* :func:`load_checkpoint` streams the shards one file at a time through
  :meth:`CausalLM.load_state_dict`, which cuts this rank's tensor-parallel slice, then folds
  the RMSNorm weights into the consuming projections once.
* :func:`save_hf_checkpoint` writes a model back in the same layout (tests, tooling).

Only safetensors are read (no pickle): the loader executes nothing from the files.
"""

from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch

from src.models.presets import ArchConfig


def is_hf_checkpoint(path: Optional[str]) -> bool:
    return bool(path) and os.path.isdir(path) and os.path.exists(os.path.join(path, "config.json")) and bool(
        glob.glob(os.path.join(path, "*.safetensors")))


def arch_from_hf_config(path: str, **overrides) -> ArchConfig:
    with open(os.path.join(path, "config.json")) as f:
        c = json.load(f)
    mt = c.get("model_type", "llama")
    if mt not in ("llama", "mistral", "mixtral"):
        raise ValueError(f"unsupported model_type {mt!r} (llama / mistral / mixtral)")
    h, nh = int(c["hidden_size"]), int(c["num_attention_heads"])
    kw = dict(
        name=os.path.basename(os.path.normpath(path)),
        hidden_size=h,
        num_layers=int(c["num_hidden_layers"]),
        num_heads=nh,
        num_kv_heads=int(c.get("num_key_value_heads") or nh),
        intermediate_size=int(c["intermediate_size"]),
        vocab_size=int(c["vocab_size"]),
        head_dim=int(c.get("head_dim") or h // nh),
        rope_theta=float(c.get("rope_theta", 10000.0)),
        rms_eps=float(c.get("rms_norm_eps", 1e-5)),
        max_position=int(c.get("max_position_embeddings", 8192)),
        num_experts=int(c.get("num_local_experts", 0)) if mt == "mixtral" else 0,
        top_k=int(c.get("num_experts_per_tok", 2)),
        tie_embeddings=bool(c.get("tie_word_embeddings", False)),
        rope_scaling=c.get("rope_scaling"),
    )
    kw.update(overrides)
    return ArchConfig(**kw)


def load_checkpoint(model, path: str) -> int:
    """Stream every ``*.safetensors`` file of ``path`` into ``model``; returns tensors loaded."""
    from safetensors import safe_open

    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    n = 0
    for fn in files:
        with safe_open(fn, framework="pt", device="cpu") as sf:
            # one shard in host memory at a time (HF shards are a few GB)
            n += model.load_state_dict({k: sf.get_tensor(k) for k in sf.keys()}, fold=False)
    model.fold_norm_weights()
    return n


def hf_state_dict(model) -> Dict[str, torch.Tensor]:
    """The model's weights under HF names (TP=1 models; norms as stored, i.e. ones once folded)."""
    if model.tp.enabled:
        raise ValueError("export a TP=1 model")
    a, d = model.arch, model.head_dim
    hq, hkv, inter = model.hq, model.hkv, model.inter
    out = {"model.embed_tokens.weight": model.embed, "model.norm.weight": model.norm,
           "lm_head.weight": model.lm_head_rows()}
    for i, lw in enumerate(model.layers):
        p = f"model.layers.{i}."
        out[p + "self_attn.q_proj.weight"] = lw.qkv[: hq * d]
        out[p + "self_attn.k_proj.weight"] = lw.qkv[hq * d:(hq + hkv) * d]
        out[p + "self_attn.v_proj.weight"] = lw.qkv[(hq + hkv) * d:]
        out[p + "self_attn.o_proj.weight"] = lw.o
        out[p + "input_layernorm.weight"] = lw.ln1
        out[p + "post_attention_layernorm.weight"] = lw.ln2
        if a.is_moe:
            out[p + "block_sparse_moe.gate.weight"] = lw.router
            for x in range(a.num_experts):
                q = p + f"block_sparse_moe.experts.{x}."
                out[q + "w1.weight"] = lw.w13[x, :inter]
                out[q + "w3.weight"] = lw.w13[x, inter:]
                out[q + "w2.weight"] = lw.w2[x]
        else:
            out[p + "mlp.gate_proj.weight"] = lw.gate_up[:inter]
            out[p + "mlp.up_proj.weight"] = lw.gate_up[inter:]
            out[p + "mlp.down_proj.weight"] = lw.down
    return out


def save_hf_checkpoint(model, path: str, shards: int = 1, overrides: Optional[Dict[str, torch.Tensor]] = None) -> None:
    """Write ``config.json`` + ``shards`` safetensors files. ``overrides`` replaces tensors by HF
    name (e.g. non-trivial norm weights for tests)."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    a = model.arch
    cfg = {"model_type": "mixtral" if a.is_moe else "llama", "hidden_size": a.hidden_size,
           "num_hidden_layers": a.num_layers, "num_attention_heads": a.num_heads,
           "num_key_value_heads": a.num_kv_heads, "intermediate_size": a.intermediate_size,
           "vocab_size": a.vocab_size, "head_dim": a.head_dim, "rope_theta": a.rope_theta,
           "rms_norm_eps": a.rms_eps, "max_position_embeddings": a.max_position,
           "tie_word_embeddings": a.tie_embeddings, "rope_scaling": a.rope_scaling}
    if a.is_moe:
        cfg.update(num_local_experts=a.num_experts, num_experts_per_tok=a.top_k)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1)
    sd = hf_state_dict(model)
    if overrides:
        sd.update(overrides)
    names = list(sd)
    per = (len(names) + shards - 1) // shards
    for s in range(shards):
        part = {k: sd[k].detach().to("cpu").contiguous() for k in names[s * per:(s + 1) * per]}
        save_file(part, os.path.join(path, f"model-{s + 1:05d}-of-{shards:05d}.safetensors"))
