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
