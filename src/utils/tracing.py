"""
Request tracing (promised at `/root/reference/README.md:18,102`; the reference
only logs durations, `src/worker.py:127-133`).

A :class:`Tracer` records per-request timelines: named *marks* (timestamps)
and *spans* (durations). The serving path stamps, per request id:

    coordinator.recv → cache_lookup → route → batch_wait → rpc → worker.recv →
    engine.queued → engine.first_token (TTFT) → engine.finished → coordinator.reply

so TTFT, TPOT (time per output token), queueing and RPC overhead come out of
one object. Traces are kept in a bounded ring and can be dumped as JSON lines.
"""

from __future__ import annotations

import contextlib
import json
import threading
import itertools
import time
import uuid
from collections import OrderedDict
from typing import Any, Dict, Iterator, List, Optional


_RID_PREFIX = uuid.uuid4().hex[:16]  # per process
_RID_SEQ = itertools.count()


def new_request_id() -> str:
    """Unique request id: a random per-process prefix + a counter (one uuid4 per request was ~10 us of the
    coordinator's per-request cost)."""
    return f"{_RID_PREFIX}{next(_RID_SEQ):016x}"


def percentile(values: List[float], q: float) -> float:
    if not values:
        return 0.0
    v = sorted(values)
    k = (len(v) - 1) * q / 100.0
    lo = int(k)
    hi = min(lo + 1, len(v) - 1)
    return v[lo] + (v[hi] - v[lo]) * (k - lo)


class Trace:
    __slots__ = ("request_id", "marks", "spans", "attrs")

    def __init__(self, request_id: str):
        self.request_id = request_id
        self.marks: Dict[str, float] = {}
        self.spans: Dict[str, float] = {}
        self.attrs: Dict[str, Any] = {}

    def to_dict(self) -> Dict[str, Any]:
        return {"request_id": self.request_id, "marks": self.marks, "spans": self.spans, "attrs": self.attrs}


class Tracer:
    """Thread-safe, bounded store of request traces."""

    def __init__(self, capacity: int = 100_000, enabled: bool = True):
        self.capacity = capacity
        self.enabled = enabled
        self._traces: "OrderedDict[str, Trace]" = OrderedDict()
        self._lock = threading.Lock()

    def _get(self, rid: str) -> Trace:
        t = self._traces.get(rid)
        if t is None:
            t = Trace(rid)
            self._traces[rid] = t
            if len(self._traces) > self.capacity:
                self._traces.popitem(last=False)
        return t

    def mark(self, rid: str, name: str, ts: Optional[float] = None) -> None:
        if not self.enabled:
            return
        with self._lock:
            self._get(rid).marks[name] = time.perf_counter() if ts is None else ts

    def add_span(self, rid: str, name: str, seconds: float) -> None:
        if not self.enabled:
            return
        with self._lock:
            t = self._get(rid)
            t.spans[name] = t.spans.get(name, 0.0) + seconds

    def set_attr(self, rid: str, key: str, value: Any) -> None:
        if not self.enabled:
            return
        with self._lock:
            self._get(rid).attrs[key] = value

    @contextlib.contextmanager
    def span(self, rid: str, name: str) -> Iterator[None]:
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.add_span(rid, name, time.perf_counter() - t0)

    def get(self, rid: str) -> Optional[Dict[str, Any]]:
        with self._lock:
            t = self._traces.get(rid)
            return t.to_dict() if t else None

    def interval(self, rid: str, start: str, end: str) -> Optional[float]:
        with self._lock:
            t = self._traces.get(rid)
            if t is None or start not in t.marks or end not in t.marks:
                return None
            return t.marks[end] - t.marks[start]

    def summary(self, start: str, end: str) -> Dict[str, float]:
        """Latency distribution (ms) of ``end - start`` over all traces having both."""
        with self._lock:
            vals = [
                (t.marks[end] - t.marks[start]) * 1e3
                for t in self._traces.values()
                if start in t.marks and end in t.marks
            ]
        return {
            "count": len(vals),
            "p50_ms": percentile(vals, 50),
            "p90_ms": percentile(vals, 90),
            "p99_ms": percentile(vals, 99),
            "mean_ms": sum(vals) / len(vals) if vals else 0.0,
        }

    def dump_jsonl(self, path: str) -> int:
        with self._lock:
            items = [t.to_dict() for t in self._traces.values()]
        with open(path, "w") as f:
            for d in items:
                f.write(json.dumps(d) + "\n")
        return len(items)

    def clear(self) -> None:
        with self._lock:
            self._traces.clear()

    def __len__(self) -> int:
        return len(self._traces)


# Process-wide default tracer.
GLOBAL_TRACER = Tracer()


def prof_marker() -> None:
    """With ``DIE_PROF_MARKERS=1``: launch one recognisable tiny kernel (torch's ``spin_kernel``) on the current
    stream. Benches bracket their timed region with two of them, and ``scripts/prof_window.py`` keeps only the
    kernels a rocprofv3 kernel trace recorded between the markers: the table then describes the timed work,
    not model init, weight packing or warm-up."""
    import os

    if os.environ.get("DIE_PROF_MARKERS") != "1":
        return
    import torch

    if torch.cuda.is_available():
        torch.cuda._sleep(1000)
