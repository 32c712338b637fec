"""Request/sequence state for the continuous-batching engine."""

from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional

from src.preproc import SamplingParams

_ids = itertools.count()


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2
    SWAPPED = 3       # preempted with its KV parked in host memory


@dataclass
class Sequence:
    request_id: str
    prompt_ids: List[int]
    sampling: SamplingParams
    on_finish: Optional[Callable[["Sequence"], None]] = None
    seq_id: int = field(default_factory=lambda: next(_ids))
    output_ids: List[int] = field(default_factory=list)
    block_table: List[int] = field(default_factory=list)
    num_computed: int = 0            # tokens whose KV is already in the cache
    num_prefix_hit: int = 0          # tokens served from the prefix cache
    block_hashes: Optional[List[int]] = None
    status: SeqStatus = SeqStatus.WAITING
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    finish_reason: Optional[str] = None
    num_preemptions: int = 0
    user_data: Any = None
    on_token: Optional[Callable[["Sequence", int], None]] = None  # streaming: called per new token
    # Disaggregation: a sequence whose prompt KV arrives from a prefill worker
    imported_kv: bool = False
    swap_buf: Any = None             # host copy of the KV blocks while SWAPPED

    def __len__(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def prompt_len(self) -> int:
        return len(self.prompt_ids)

    @property
    def in_prefill(self) -> bool:
        return self.num_computed < self.prompt_len

    @property
    def last_token(self) -> int:
        return self.output_ids[-1] if self.output_ids else self.prompt_ids[-1]

    def token_at(self, i: int) -> int:
        p = self.prompt_len
        return self.prompt_ids[i] if i < p else self.output_ids[i - p]

    def ttft_ms(self) -> Optional[float]:
        return None if self.first_token_time is None else (self.first_token_time - self.arrival) * 1e3

    def latency_ms(self) -> Optional[float]:
        return None if self.finish_time is None else (self.finish_time - self.arrival) * 1e3
