#!/usr/bin/env python3
"""Batcher behaviour (the reference's examples/batcher_demo.py scenarios, re-done):
size-triggered flushes, latency-triggered flushes, and streaming completion."""

import asyncio
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.batcher import Batcher  # noqa: E402
from src.mock_models import mock_batch_inference  # noqa: E402


async def scenario(title, max_batch, max_latency_ms, n, spacing_s):
    sizes = []

    async def cb(m, v, xs):
        sizes.append(len(xs))
        return await mock_batch_inference(m, v, xs, latency_ms=20)

    b = Batcher(max_batch_size=max_batch, max_latency_ms=max_latency_ms, batch_callback=cb)
    await b.start()
    t0 = time.perf_counter()
    futs = []
    for i in range(n):
        futs.append(await b.add_request("demo", "1", f"req-{i}"))
        await asyncio.sleep(spacing_s)
    res = await asyncio.gather(*futs)
    await b.stop()
    st = await b.get_stats()
    print(f"{title}: batches {sizes} (avg {st['avg_batch_size']:.2f}), {sum(r['success'] for r in res)}/{n} ok, "
          f"{1e3 * (time.perf_counter() - t0):.0f} ms, pending {st['pending_batches_count']}")


async def main():
    await scenario("size flush   (batch 5, 500 ms, 12 reqs @ 5 ms)", 5, 500, 12, 0.005)
    await scenario("latency flush(batch 10, 20 ms, 3 reqs @ 50 ms)", 10, 20, 3, 0.05)
    await scenario("config-2 knob(batch 32, 10 ms, 100 reqs @ 0)", 32, 10, 100, 0)


if __name__ == "__main__":
    asyncio.run(main())
