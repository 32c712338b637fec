"""Model families: Llama-3 (dense) and Mixtral (MoE) decoders on the gfx950 kernels."""

from .llama import AttnMetadata, CausalLM  # noqa: F401
from .presets import PRESETS, ArchConfig, get_preset  # noqa: F401
