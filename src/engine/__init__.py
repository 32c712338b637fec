"""Serving engine: paged KV blocks (native block manager), continuous-batching
scheduler, hipGraph decode runner, async front for the worker."""

from .llm_engine import LLMEngine  # noqa: F401
from .sequence import Sequence, SeqStatus  # noqa: F401
