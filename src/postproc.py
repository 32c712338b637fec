"""
Post-processing: detokenisation and response shaping
(promised at `/root/reference/README.md:35,96-98`, absent from the reference).
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional


def build_llm_output(token_ids: List[int], tokenizer=None, *, prompt_len: int, finish_reason: str,
                     ttft_ms: Optional[float] = None, latency_ms: Optional[float] = None,
                     return_text: bool = True) -> Dict[str, Any]:
    out: Dict[str, Any] = {
        "token_ids": list(token_ids),
        "num_prompt_tokens": prompt_len,
        "num_output_tokens": len(token_ids),
        "finish_reason": finish_reason,
    }
    if return_text and tokenizer is not None:
        out["text"] = tokenizer.decode(token_ids)
    if ttft_ms is not None:
        out["ttft_ms"] = ttft_ms
    if latency_ms is not None:
        out["latency_ms"] = latency_ms
        n = len(token_ids)
        if ttft_ms is not None and n > 1:
            out["tpot_ms"] = (latency_ms - ttft_ms) / (n - 1)
    return out


def postprocess(outputs: Any) -> Any:
    """Generic hook for non-LLM outputs (identity unless a dict of floats,
    which are rounded for transport)."""
    if isinstance(outputs, dict):
        return {k: (round(v, 6) if isinstance(v, float) else v) for k, v in outputs.items()}
    return outputs
