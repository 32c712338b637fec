"""
Architecture presets (shapes only — weights are random-initialised on device
unless a local safetensors checkpoint is given; there is no network here).

Shapes from the public model cards: Llama-3-8B / 70B (GQA 8 kv heads,
RoPE θ=500000, vocab 128256) and Mixtral-8x7B (8 experts, top-2, θ=1e6,
vocab 32000). SURVEY §2F lists them as the BASELINE configs.
"""

from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Any, Dict, Optional


@dataclass(frozen=True)
class ArchConfig:
    name: str
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    intermediate_size: int
    vocab_size: int
    head_dim: int = 128
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    num_experts: int = 0          # 0 → dense MLP
    top_k: int = 2
    tie_embeddings: bool = False
    rope_scaling: Optional[Dict[str, Any]] = field(default=None, hash=False, compare=False)

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def param_count(self) -> int:
        h, i, l = self.hidden_size, self.intermediate_size, self.num_layers
        attn = h * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim + self.num_heads * self.head_dim * h
        mlp = 3 * h * i * max(1, self.num_experts) + (h * self.num_experts if self.is_moe else 0)
        emb = self.vocab_size * h * (1 if self.tie_embeddings else 2)
        return l * (attn + mlp + 2 * h) + emb + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.num_kv_heads * self.head_dim * dtype_bytes


PRESETS: Dict[str, ArchConfig] = {
    "llama3-8b": ArchConfig("llama3-8b", 4096, 32, 32, 8, 14336, 128256, rope_theta=500000.0),
    "llama3-70b": ArchConfig("llama3-70b", 8192, 80, 64, 8, 28672, 128256, rope_theta=500000.0),
    "mixtral-8x7b": ArchConfig("mixtral-8x7b", 4096, 32, 32, 8, 14336, 32000, rope_theta=1e6,
                               max_position=32768, num_experts=8, top_k=2),
    # small shapes for tests / smoke (same kernels, same code paths)
    "llama-tiny": ArchConfig("llama-tiny", 256, 2, 4, 2, 512, 1024, max_position=2048),
    "llama-mini": ArchConfig("llama-mini", 1024, 4, 8, 2, 2048, 32000, max_position=4096),
    "mixtral-tiny": ArchConfig("mixtral-tiny", 256, 2, 4, 2, 256, 1024, rope_theta=1e6, max_position=2048,
                               num_experts=4, top_k=2),
}


def get_preset(name: str, **overrides) -> ArchConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; known: {sorted(PRESETS)}")
    cfg = PRESETS[name]
    return replace(cfg, **overrides) if overrides else cfg
