"""Batcher: flush on size and on latency, per-key batching, error fan-out,
streaming completion, no deadlock on re-entry, drain on stop."""

import asyncio

import pytest

from src.batcher import Batcher
from src.mock_models import mock_batch_inference


def run(coro):
    return asyncio.run(coro)


def test_size_and_latency_flush():
    async def main():
        sizes = []

        async def cb(m, v, xs):
            sizes.append(len(xs))
            return await mock_batch_inference(m, v, xs, latency_ms=5)

        b = Batcher(max_batch_size=5, max_latency_ms=80, batch_callback=cb)
        await b.start()
        futs = []
        for i in range(12):
            futs.append(await b.add_request("m", "1", i))
            await asyncio.sleep(0.002)
        res = await asyncio.gather(*futs)
        await b.stop()
        assert sizes == [5, 5, 2]
        assert [r["input_id"] for r in res] == [0, 1, 2, 3, 4] * 2 + [0, 1]
        st = await b.get_stats()
        assert st["total_batches"] == 3 and st["total_requests"] == 12 and st["avg_batch_size"] == 4
    run(main())


def test_add_request_does_not_wait_for_model():
    async def main():
        async def slow(m, v, xs):
            await asyncio.sleep(0.3)
            return xs

        b = Batcher(max_batch_size=1, max_latency_ms=1000, batch_callback=slow)
        await b.start()
        t0 = asyncio.get_running_loop().time()
        fut = await b.add_request("m", "1", "x")
        assert asyncio.get_running_loop().time() - t0 < 0.1
        assert await fut == "x"
        await b.stop()
    run(main())


def test_keys_are_batched_separately():
    async def main():
        seen = []

        async def cb(m, v, xs):
            seen.append((m, v, sorted(xs)))
            return xs

        b = Batcher(max_batch_size=10, max_latency_ms=20, batch_callback=cb)
        await b.start()
        fs = [await b.add_request("a", "1", 1), await b.add_request("b", "1", 2), await b.add_request("a", "1", 3)]
        await asyncio.gather(*fs)
        await b.stop()
        assert sorted(seen) == [("a", "1", [1, 3]), ("b", "1", [2])]
    run(main())


def test_errors_fan_out_and_no_callback():
    async def main():
        async def bad(m, v, xs):
            raise RuntimeError("boom")

        b = Batcher(max_batch_size=2, max_latency_ms=10, batch_callback=bad)
        await b.start()
        fs = [await b.add_request("m", "1", i) for i in range(2)]
        for f in fs:
            with pytest.raises(RuntimeError):
                await f
        await b.stop()
        b2 = Batcher(max_batch_size=1, max_latency_ms=10)
        await b2.start()
        with pytest.raises(RuntimeError):
            await (await b2.add_request("m", "1", 0))
        await b2.stop()
        with pytest.raises(RuntimeError):
            await b2.add_request("m", "1", 0)
    run(main())


def test_reentrant_callback_does_not_deadlock():
    async def main():
        b = None

        async def cb(m, v, xs):
            if m == "outer":
                inner = await b.add_request("inner", "1", "y")
                return [await asyncio.wait_for(inner, 2.0) for _ in xs]
            return [x + "!" for x in xs]

        b = Batcher(max_batch_size=8, max_latency_ms=10, batch_callback=cb)
        await b.start()
        r = await asyncio.wait_for(await b.add_request("outer", "1", "x"), 3.0)
        assert r == "y!"
        await b.stop()
    run(main())


def test_streaming_completion():
    async def main():
        async def cb(m, v, xs):
            async def one(x):
                await asyncio.sleep(0.01 * x)
                return x * 10
            return [one(x) for x in xs]

        b = Batcher(max_batch_size=3, max_latency_ms=50, batch_callback=cb)
        await b.start()
        fs = [await b.add_request("m", "1", x) for x in (1, 20, 2)]
        done, _ = await asyncio.wait(fs, timeout=0.1)
        assert {f.result() for f in done} == {10, 20}  # the slow one is not waited for
        assert await fs[1] == 200
        await b.stop()
    run(main())


def test_stop_drains_pending():
    async def main():
        async def cb(m, v, xs):
            return xs

        b = Batcher(max_batch_size=100, max_latency_ms=10_000, batch_callback=cb)
        await b.start()
        f = await b.add_request("m", "1", "pending")
        await b.stop()
        assert f.result() == "pending"
    run(main())


def test_coalesce_split():
    async def main():
        async def cb(m, v, payload):
            return payload.upper()

        b = Batcher(max_batch_size=3, max_latency_ms=10, batch_callback=cb,
                    coalesce=lambda xs: "|".join(xs), split=lambda out, n: out.split("|"))
        await b.start()
        fs = [await b.add_request("m", "1", s) for s in ("a", "b", "c")]
        assert await asyncio.gather(*fs) == ["A", "B", "C"]
        await b.stop()
    run(main())


def test_validation():
    with pytest.raises(ValueError):
        Batcher(max_batch_size=0)
    with pytest.raises(ValueError):
        Batcher(max_latency_ms=0)


def test_idle_gap_flush_does_not_wait_max_latency():
    """idle_flush_ms: a partial batch goes out once arrivals pause (closed-loop clients all waiting on it),
    long before max_latency; a steady stream of arrivals still batches up to max_latency / max_batch."""
    import asyncio
    import time

    from src.batcher import Batcher

    async def main():
        sizes = []

        async def cb(model, version, inputs):
            sizes.append(len(inputs))
            return inputs

        b = Batcher(max_batch_size=32, max_latency_ms=200.0, batch_callback=cb, idle_flush_ms=2.0)
        await b.start()
        t0 = time.perf_counter()
        futs = [await b.add_request("m", "1", i) for i in range(5)]
        await asyncio.gather(*futs)
        quick = time.perf_counter() - t0
        t0 = time.perf_counter()
        futs = []
        for i in range(10):  # arrivals 1 ms apart: under the idle gap, so they keep batching
            futs.append(await b.add_request("m", "1", i))
            await asyncio.sleep(0.001)
        await asyncio.gather(*futs)
        await b.stop()
        return quick, sizes

    quick, sizes = asyncio.run(main())
    assert quick < 0.1, quick          # not the 200 ms max_latency
    assert sizes[0] == 5 and sum(sizes) == 15 and max(sizes[1:]) >= 5, sizes
