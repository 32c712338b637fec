#!/usr/bin/env python3
"""Start a worker in-process and talk to it (mock echo model by default, or a
real Llama session with --arch llama --preset llama-mini on a GPU)."""

import argparse
import asyncio
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.client import InferenceClient  # noqa: E402
from src.config import ModelConfig  # noqa: E402
from src.worker import Worker  # noqa: E402


async def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mock")
    ap.add_argument("--preset", default="llama-mini")
    a = ap.parse_args()
    w = Worker("demo-worker", host="127.0.0.1", install_signal_handlers=False)
    cfg = ModelConfig("demo", "", batch_size=8, max_batch_size=32, input_schema={"input": "string"},
                      arch=a.arch, preset=a.preset, max_model_len=1024)
    assert w.load_model(cfg)
    port = await w.start()
    c = InferenceClient(f"127.0.0.1:{port}")
    inputs = {"prompt": "The MI355X has", "max_tokens": 8} if a.arch != "mock" else {"input": "hello"}
    print(json.dumps(await c.call({"model": "demo", "inputs": inputs}), indent=2))
    print(json.dumps((await c.call({"op": "metrics"}))["metrics"], indent=2, default=str)[:2000])
    c.close()
    await w.shutdown()


if __name__ == "__main__":
    asyncio.run(main())
