#!/usr/bin/env python3
"""Send requests to a coordinator (or a worker) and print the replies.

    python examples/example_client.py --address 127.0.0.1:9000 --model echo --inputs '{"x": 1}'
    python examples/example_client.py --model llama --prompt "Hello" --max-tokens 32
    python examples/example_client.py --model llama --prompt "Hi" -n 64 --concurrency 32   # mini load test
    python examples/example_client.py --model llama --prompt "Hello" --max-tokens 64 --stream  # token stream
"""

import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.client import InferenceClient  # noqa: E402
from src.utils import percentile  # noqa: E402


async def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", default="127.0.0.1:9000")
    ap.add_argument("--model", default="echo")
    ap.add_argument("--inputs", default=None, help="raw JSON inputs (mock models)")
    ap.add_argument("--prompt", default=None)
    ap.add_argument("--max-tokens", type=int, default=16)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--request-key", default=None, help="session key for shard affinity")
    ap.add_argument("-n", type=int, default=1)
    ap.add_argument("--concurrency", type=int, default=1)
    ap.add_argument("--poll", action="store_true", help="submit + poll instead of waiting")
    ap.add_argument("--stream", action="store_true", help="print token deltas as they are generated")
    a = ap.parse_args()
    if a.prompt is not None:
        inputs = {"prompt": a.prompt, "max_tokens": a.max_tokens, "temperature": a.temperature}
    else:
        inputs = json.loads(a.inputs) if a.inputs else {"text": "hello"}
    c = InferenceClient(a.address)
    if a.stream:
        t0 = time.perf_counter()
        async for frame in c.infer_stream(a.model, inputs, request_key=a.request_key):
            if frame.get("done") is False:
                print(f"[{1e3 * (time.perf_counter() - t0):8.1f} ms] +{frame['delta_token_ids']}", flush=True)
            else:
                print(json.dumps(frame, indent=2)[:4000])
        c.close()
        return
    sem = asyncio.Semaphore(a.concurrency)
    lat = []

    async def one(i):
        async with sem:
            t0 = time.perf_counter()
            if a.poll:
                rid = await c.submit(a.model, inputs)
                r = await c.result(rid)
            else:
                r = await c.infer(a.model, inputs, request_key=a.request_key, cache=a.n == 1)
            lat.append(time.perf_counter() - t0)
            return r

    t0 = time.perf_counter()
    rs = await asyncio.gather(*(one(i) for i in range(a.n)))
    el = time.perf_counter() - t0
    if a.n == 1:
        print(json.dumps(rs[0], indent=2)[:4000])
    else:
        ok = sum(1 for r in rs if r.get("success"))
        print(f"{ok}/{a.n} ok, {a.n / el:.1f} req/s, p50 {1e3 * percentile(lat, 50):.1f} ms, "
              f"p99 {1e3 * percentile(lat, 99):.1f} ms")
    c.close()


if __name__ == "__main__":
    asyncio.run(main())
