#!/usr/bin/env python3
"""Start a worker in-process and talk to it over its RPC port (mock echo model by
default, or a real Llama session with --arch llama --preset llama-mini on a GPU).

    python examples/worker_demo.py                 # one request + metrics, then exit
    python examples/worker_demo.py --interactive   # REPL: predict <text|json> / metrics / models / help / exit

The REPL keeps the reference demo's commands (`/root/reference/examples/worker_demo.py:125-217`)
but sends every request through the worker's TCP server instead of calling it in-process.
"""

import argparse
import asyncio
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.client import InferenceClient  # noqa: E402
from src.config import ModelConfig  # noqa: E402
from src.worker import Worker  # noqa: E402


HELP = """predict <text or JSON inputs>   run one request (LLM: text is the prompt)
metrics                         worker metrics (requests, errors, memory, model stats)
models                          loaded models
help                            this text
exit                            stop the worker and quit"""


async def repl(c, arch):
    loop = asyncio.get_running_loop()
    print(HELP)
    while True:
        try:
            line = (await loop.run_in_executor(None, input, "worker> ")).strip()
        except (EOFError, KeyboardInterrupt):
            break
        cmd, _, arg = line.partition(" ")
        if cmd in ("exit", "quit"):
            break
        if cmd == "help" or not cmd:
            print(HELP)
        elif cmd == "predict":
            try:
                inputs = json.loads(arg)
            except ValueError:
                inputs = {"prompt": arg, "max_tokens": 16} if arch != "mock" else {"input": arg}
            print(json.dumps(await c.call({"model": "demo", "inputs": inputs}), indent=2, default=str))
        elif cmd == "metrics":
            print(json.dumps((await c.call({"op": "metrics"}))["metrics"], indent=2, default=str))
        elif cmd == "models":
            print(json.dumps((await c.call({"op": "health"})).get("models"), indent=2))
        else:
            print(f"unknown command {cmd!r}; try help")


async def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mock")
    ap.add_argument("--preset", default="llama-mini")
    ap.add_argument("--interactive", action="store_true")
    a = ap.parse_args()
    w = Worker("demo-worker", host="127.0.0.1", install_signal_handlers=False)
    cfg = ModelConfig("demo", "", batch_size=8, max_batch_size=32, input_schema={"input": "string"},
                      arch=a.arch, preset=a.preset, max_model_len=1024)
    assert w.load_model(cfg)
    port = await w.start()
    c = InferenceClient(f"127.0.0.1:{port}")
    if a.interactive:
        await repl(c, a.arch)
        c.close()
        await w.shutdown()
        return
    inputs = {"prompt": "The MI355X has", "max_tokens": 8} if a.arch != "mock" else {"input": "hello"}
    print(json.dumps(await c.call({"model": "demo", "inputs": inputs}), indent=2))
    print(json.dumps((await c.call({"op": "metrics"}))["metrics"], indent=2, default=str)[:2000])
    c.close()
    await w.shutdown()


if __name__ == "__main__":
    asyncio.run(main())
