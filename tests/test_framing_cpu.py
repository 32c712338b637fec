"""Legacy (unframed JSON) request reader: the end of the top-level object is found by one incremental scan
(src/utils/framing.py), not by re-decoding the whole buffer after every chunk (quadratic)."""

import asyncio
import json
import random
import time

from src.utils.framing import _JsonObjectEnd, read_legacy_json


async def _read(data: bytes, chunk: int):
    r = asyncio.StreamReader()
    for i in range(1, len(data), chunk):
        r.feed_data(data[i:i + chunk])
    r.feed_eof()
    return await read_legacy_json(r, data[:1])


def test_escape_across_chunk_boundary():
    sc = _JsonObjectEnd()
    parts = [b'{"a":"x\\', b'"}', b'"}']  # the escaped quote starts a new chunk
    ends, base = [], 0
    for p in parts:
        ends.append(sc.feed(p, base))
        base += len(p)
    assert ends == [-1, -1, 12]


def test_random_documents_any_chunking():
    rng = random.Random(1)
    alphabet = 'ab{}[]"\\ ,:'
    for _ in range(300):
        d = {f"k{i}": "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 12)))
             for i in range(rng.randint(1, 5))}
        d["n"] = [rng.randint(0, 9), {"x": '}]\\"'}]
        data = json.dumps(d).encode()
        for ch in (1, 2, 3, 5, 64):
            assert asyncio.run(_read(data, ch)) == d


def test_trailing_bytes_after_object_are_ignored():
    assert asyncio.run(_read(b'{"a": 1}   \n', 4)) == {"a": 1}


def test_large_document_is_linear():
    data = json.dumps({"inputs": "q" * 8_000_000}).encode()
    t = time.perf_counter()
    assert len(asyncio.run(_read(data, 65536))["inputs"]) == 8_000_000
    assert time.perf_counter() - t < 5.0  # the quadratic reader took minutes at this size


# --------------------------------------------------------------------------- ADVICE r4 (frame server)
def test_pipelining_client_is_backpressured_and_fully_served():
    """A client that pipelines far more frames than the server serves at once: the protocol stops reading
    (pause_reading) once MAX_QUEUED decoded requests wait, so the queue never grows past that bound, and every
    request is still answered, in order, once the handler drains."""
    from src.utils.frameserver import FrameServerProtocol
    from src.utils.framing import _HDR, deserialize, pack_frame

    async def main():
        gate = asyncio.Event()
        protos, peak = [], [0]

        async def handler(msg, emit):
            await gate.wait()
            peak[0] = max(peak[0], len(protos[0]._queue))
            return {"i": msg["i"]}

        loop = asyncio.get_running_loop()

        def factory():
            p = FrameServerProtocol(handler)
            protos.append(p)
            return p

        srv = await loop.create_server(factory, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        r, w = await asyncio.open_connection("127.0.0.1", port)
        n = 400
        w.write(b"".join(pack_frame({"i": i, "pad": "x" * 2000}) for i in range(n)))
        await asyncio.sleep(0.3)  # the server reads until its queue is full, then pauses
        queued = len(protos[0]._queue)
        paused = protos[0]._reading_paused
        gate.set()
        got = []
        for _ in range(n):
            hdr = await asyncio.wait_for(r.readexactly(4), 10)
            (ln,) = _HDR.unpack(hdr)
            got.append(deserialize(await r.readexactly(ln))["i"])
        w.close()
        srv.close()
        return queued, paused, peak[0], got

    queued, paused, peak, got = asyncio.run(main())
    assert paused and queued <= FrameServerProtocol.MAX_QUEUED
    assert peak <= FrameServerProtocol.MAX_QUEUED
    assert got == list(range(400))


def test_worker_counts_protocol_rejects_as_errors():
    """A malformed frame rejected by the framing layer is counted in the worker's metrics (request_count and
    error_count), as the reference counted a request that failed to decode."""
    from src.worker import Worker

    async def main():
        w = Worker("w-err", host="127.0.0.1", port=0, install_signal_handlers=False)
        port = await w.start()
        r, wr = await asyncio.open_connection("127.0.0.1", port)
        wr.write(b"\xff\xff\xff\xff" + b"junk")  # frame length beyond MAX_FRAME
        await asyncio.wait_for(r.read(), 5)     # the error reply, then the server closes the connection
        wr.close()
        m = w.get_metrics()
        await w.shutdown()
        return m

    m = asyncio.run(main())
    assert m["error_count"] == 1 and m["request_count"] == 1
