"""
Batch mock with fault injection (`/root/reference/src/mock_models/mock_inference.py:12-73`):
sleeps ``latency_ms`` once per batch and returns one result per input; the first
``ceil(error_rate * N)`` inputs fail.
"""

import asyncio
import logging
import time
from typing import Any, Dict, List

logger = logging.getLogger(__name__)


async def mock_batch_inference(model_name: str, version: str, inputs: List[Any], **kwargs) -> List[Dict[str, Any]]:
    latency_ms = kwargs.get("latency_ms", 100)
    error_rate = kwargs.get("error_rate", 0.0)
    n = len(inputs)
    t0 = time.time()
    if latency_ms > 0:
        await asyncio.sleep(latency_ms / 1000.0)
    out: List[Dict[str, Any]] = []
    for i, x in enumerate(inputs):
        if error_rate > 0 and (i / n) < error_rate:
            out.append({"success": False, "error": f"Simulated error processing input {i}",
                        "model": model_name, "version": version, "input_id": i})
        else:
            out.append({"success": True, "result": f"Processed by {model_name}:{version} - {x}",
                        "model": model_name, "version": version, "input_id": i,
                        "metadata": {"processing_time_ms": latency_ms, "batch_size": n,
                                     "batch_position": i, "timestamp": time.time()}})
    logger.debug("Processed batch of %d in %.2fms", n, (time.time() - t0) * 1e3)
    return out
