"""
Echo model with simulated latency (`/root/reference/src/mock_models/fake_model.py:11-83`).

Behaviour kept: ``predict`` sleeps and echoes ``{"model","output","metadata"}``.
Changes: the simulated latency is configurable (``latency_s``; default keeps
the reference's pseudo-random 50–150 ms, ``0`` measures pure plumbing), the
request id is collision-free, ``predict_batch`` serves a whole batch in one
sleep, and ``get_metrics`` reports latency in both seconds and milliseconds
(the reference's REPL printed seconds as ms).
"""

import asyncio
import itertools
import time
import uuid
from typing import Any, Dict, List, Optional

from src.config import ModelConfig

_seq = itertools.count()
_PREFIX = uuid.uuid4().hex[:12]  # per process: ids stay collision-free across workers without a uuid per request


class FakeModel:
    def __init__(self, config: ModelConfig, latency_s: Optional[float] = None):
        self.config = config
        self.model_name = config.model_name
        self.batch_size = config.batch_size
        self.max_batch_size = config.max_batch_size
        self.input_schema = config.input_schema or {}
        self.output_schema = config.output_schema or {}
        if latency_s is None:
            latency_s = config.overrides.get("latency_s") if config.overrides else None
        self.latency_s = latency_s  # None → reference 50-150 ms pseudo-random
        self.request_count = 0
        self.error_count = 0
        self.total_latency = 0.0
        self.last_inference_time = 0.0

    def _sleep_time(self) -> float:
        if self.latency_s is None:
            return 0.05 + (time.time() % 0.1)
        return float(self.latency_s)

    def _result(self, inputs: Any, batch_size: int) -> Dict[str, Any]:
        return {
            "model": self.model_name,
            "output": inputs,
            "metadata": {
                "batch_size": batch_size,
                "timestamp": time.time(),
                "request_id": f"req_{_PREFIX}_{next(_seq)}",
            },
        }

    async def predict(self, inputs: Any) -> Dict[str, Any]:
        t0 = time.time()
        self.request_count += 1
        try:
            d = self._sleep_time()
            if d > 0:
                await asyncio.sleep(d)
            return self._result(inputs, len(inputs) if isinstance(inputs, (list, tuple)) else 1)
        except Exception:
            self.error_count += 1
            raise
        finally:
            self.total_latency += time.time() - t0
            self.last_inference_time = time.time()

    async def predict_batch(self, inputs_list: List[Any]) -> List[Dict[str, Any]]:
        t0 = time.time()
        self.request_count += len(inputs_list)
        d = self._sleep_time()
        if d > 0:
            await asyncio.sleep(d)
        out = [self._result(x, len(inputs_list)) for x in inputs_list]
        self.total_latency += (time.time() - t0) * len(inputs_list)
        self.last_inference_time = time.time()
        return out

    def get_metrics(self) -> Dict[str, Any]:
        avg = (self.total_latency / self.request_count) if self.request_count else 0.0
        return {
            "model_name": self.model_name,
            "request_count": self.request_count,
            "error_count": self.error_count,
            "avg_latency": avg,
            "avg_latency_ms": avg * 1e3,
            "last_inference_time": self.last_inference_time,
            "batch_size": self.batch_size,
            "max_batch_size": self.max_batch_size,
        }

    def close(self) -> None:
        pass
