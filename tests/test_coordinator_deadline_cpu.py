"""Coordinator dispatch bounds: the retries of one request share ONE deadline
(request_timeout_s), on the direct (lone request) path as on the batch path, and a direct dispatch
counts against the batcher's max_inflight_batches."""

import asyncio
import time

from src.batcher import Batcher
from src.coordinator import Coordinator


def test_send_retries_share_one_deadline():
    async def main():
        coord = Coordinator(port=0, request_timeout_s=0.3, max_retries=5)
        calls = []

        async def hang(addr, msg, timeout=None):
            calls.append(timeout)
            await asyncio.sleep(timeout)
            raise asyncio.TimeoutError()

        coord._candidates = lambda *a: [(f"w{i}", f"127.0.0.1:{9 + i}") for i in range(6)]
        coord.rpc.call = hang
        t0 = time.monotonic()
        rep = await coord._send("m", "1", 0, "k", {"op": "infer"}, deadline=time.monotonic() + 0.3)
        dt = time.monotonic() - t0
        assert not rep["success"]
        assert dt < 0.6, dt  # was up to (max_retries + 1) x request_timeout_s
        assert sum(calls) <= 0.31 + 1e-6, calls
    asyncio.run(main())


def test_direct_dispatch_respects_inflight_limit():
    async def main():
        async def cb(model, version, items):
            await asyncio.sleep(0.05)
            return items

        b = Batcher(max_batch_size=4, max_latency_ms=5, batch_callback=cb, max_inflight_batches=1,
                    eager_when_idle=True)
        await b.start()
        assert b.try_direct("m", "a")          # takes the only in-flight slot
        assert not b.try_direct("m", "b")      # another key: no slot left, it must queue
        fut = await b.add_request("m", "b", 1)
        await asyncio.sleep(0.03)
        assert not fut.done()                  # its batch waits for the slot held by the direct request
        b.release_direct("m", "a")
        assert await asyncio.wait_for(fut, 1.0) == 1
        assert b.try_direct("m", "a")
        b.release_direct("m", "a")
        await b.stop()
    asyncio.run(main())
