"""End-to-end control plane on CPU (BASELINE config 1): coordinator + 2 mock
workers as separate processes, framed and legacy wire formats, caching,
batching, polling, registration handshake and failover when a worker dies."""

import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time

import pytest

from src.client import InferenceClient, legacy_request
from src.coordinator import Coordinator
from src.utils import deserialize, pack_frame, serialize, CODEC_MSGPACK, ProtocolError
from src.worker import Worker
from src.config import ModelConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def spawn_worker(wid, coordinator=None, latency_ms=5):
    fd, pf = tempfile.mkstemp()
    os.close(fd)
    os.unlink(pf)
    cmd = [sys.executable, "-m", "src.worker", "--worker-id", wid, "--host", "127.0.0.1", "--port", "0",
           "--model", "echo", "--arch", "mock", "--mock-latency-ms", str(latency_ms), "--port-file", pf]
    if coordinator:
        cmd += ["--coordinator", coordinator]
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for _ in range(200):
        if os.path.exists(pf):
            with open(pf) as f:
                port = int(f.read())
            os.unlink(pf)
            return p, f"127.0.0.1:{port}"
        time.sleep(0.05)
    p.kill()
    raise RuntimeError("worker did not start")


def test_framing_roundtrip():
    obj = {"a": [1, 2, {"b": "x" * 10000}]}
    assert deserialize(serialize(obj)) == obj
    assert deserialize(serialize(obj, CODEC_MSGPACK)) == obj
    with pytest.raises(ProtocolError):
        deserialize(b"P" + b"junk")           # pickle refused by default
    assert pack_frame(obj)[:4] == len(serialize(obj)).to_bytes(4, "big")


def test_read_message_large_frame_lengths_are_not_legacy():
    """Frame lengths whose high byte is 0x09/0x0A/0x0D/0x20 (144-528 MiB, e.g. a 4K-token
    kv_import) must be parsed as frames, never as legacy JSON (framing.py:126)."""
    from src.utils.framing import read_message

    async def main():
        for n in (0x20000000, 0x09000000, 0x0A000010, 0x0D000000):
            r = asyncio.StreamReader()
            # header only + EOF: a framed parse must try to read n bytes and fail with
            # IncompleteReadError; the old legacy path returned/raised JSON errors instead
            r.feed_data(n.to_bytes(4, "big") + b"J{}")
            r.feed_eof()
            with pytest.raises(asyncio.IncompleteReadError):
                await read_message(r)
        r = asyncio.StreamReader()
        r.feed_data(b'{"model": "echo"}')
        r.feed_eof()
        obj, mode, _ = await read_message(r)
        assert mode == "legacy" and obj == {"model": "echo"}
        r = asyncio.StreamReader()
        r.feed_data(pack_frame({"op": "health"}))
        r.feed_eof()
        obj, mode, _ = await read_message(r)
        assert mode == "framed" and obj == {"op": "health"}

    asyncio.run(main())


def test_in_process_worker_api():
    async def main():
        w = Worker("w", host="127.0.0.1", install_signal_handlers=False)
        assert w.load_model(ModelConfig("echo", "/x", arch="mock", overrides={"latency_s": 0}))
        r = await w._process_request({"model": "echo", "inputs": {"x": 1}})
        assert r["success"] and r["outputs"]["output"] == {"x": 1} and r["worker_id"] == "w"
        assert not (await w._process_request({"model": "nope", "inputs": 1}))["success"]
        assert not (await w._process_request({"inputs": 1}))["success"]
        port = await w.start()
        big = "y" * 100_000                       # > 4 KiB: the reference's read(4096) broke here
        r = await legacy_request(f"127.0.0.1:{port}", {"model": "echo", "inputs": big})
        assert r["success"] and r["outputs"]["output"] == big
        c = InferenceClient(f"127.0.0.1:{port}")
        for i in range(5):                        # persistent framed connection
            r = await c.call({"model": "echo", "inputs": i})
            assert r["outputs"]["output"] == i
        h = await c.call({"op": "health"})
        assert h["success"] and h["models"] == ["echo"]
        m = (await c.call({"op": "metrics"}))["metrics"]
        assert m["request_count"] == 6 and m["probe_count"] == 1
        c.close()
        await w.shutdown()
    asyncio.run(main())


def test_coordinator_two_workers_end_to_end():
    async def main():
        coord = Coordinator(port=0, max_batch_size=8, max_latency_ms=5, health_check_interval=0.2)
        cport = await coord.start()
        caddr = f"127.0.0.1:{cport}"
        procs = []
        try:
            for i in range(2):
                procs.append(spawn_worker(f"w{i}", coordinator=caddr))
            for _ in range(200):
                if coord.healthy_worker_count() == 2:
                    break
                await asyncio.sleep(0.05)
            assert coord.healthy_worker_count() == 2
            client = InferenceClient(caddr)
            rs = await asyncio.gather(*(client.infer("echo", {"i": i}, cache=False) for i in range(64)))
            assert all(r["success"] for r in rs)
            assert [r["outputs"]["output"]["i"] for r in rs] == list(range(64))
            assert {r["worker_id"] for r in rs} == {"w0", "w1"}       # both shards used
            # cache: second identical request is a hit
            a = await client.infer("echo", "same")
            b = await client.infer("echo", "same")
            assert not a.get("cached") and b.get("cached")
            # request_key affinity
            ws = {(await client.infer("echo", j, request_key="user-42", cache=False))["worker_id"] for j in range(5)}
            assert len(ws) == 1
            # polling mode
            rid = await client.submit("echo", "later")
            res = await client.result(rid, timeout=10)
            assert res["success"] and res["outputs"]["output"] == "later"
            # unknown model
            assert not (await client.infer("nope", 1))["success"]
            # legacy unframed client against the coordinator
            r = await legacy_request(caddr, {"model": "echo", "inputs": "legacy"})
            assert r["success"]
            st = (await client.stats())["stats"]
            assert st["batcher"]["avg_batch_size"] > 1.0
            # kill the worker that owns user-42: requests fail over to the survivor
            victim = next(iter(ws))
            idx = int(victim[1:])
            procs[idx][0].kill()
            procs[idx][0].wait()
            rs = await asyncio.gather(*(client.infer("echo", k, request_key="user-42", cache=False)
                                        for k in range(10)))
            assert all(r["success"] for r in rs)
            assert {r["worker_id"] for r in rs} == {f"w{1 - idx}"}
            client.close()
        finally:
            for p, _ in procs:
                p.kill()
                p.wait()
            await coord.stop()
    asyncio.run(main())


def test_multi_process_coordinator_shares_port_and_forwards_registration(tmp_path):
    """--procs 3: three coordinator processes on one SO_REUSEPORT port; a worker registers with
    whichever accepts its connection and the registration is forwarded to the siblings, so requests
    on any connection (spread by the kernel) are served."""
    import os
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pf = str(tmp_path / "coord.port")
    coord = subprocess.Popen([sys.executable, "-m", "src.coordinator", "--listen-port", "0", "--procs", "3",
                              "--port-file", pf], cwd=root, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    worker = None
    try:
        t0 = time.time()
        while not os.path.exists(pf):
            assert coord.poll() is None and time.time() - t0 < 60, "coordinators did not start"
            time.sleep(0.1)
        cport = int(open(pf).read())
        wpf = str(tmp_path / "w.port")
        worker = subprocess.Popen([sys.executable, "-m", "src.worker", "--worker-id", "w-mp", "--host", "127.0.0.1",
                                   "--port", "0", "--port-file", wpf, "--model", "echo", "--arch", "mock",
                                   "--mock-latency-ms", "0", "--coordinator", f"127.0.0.1:{cport}"],
                                  cwd=root, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        while not os.path.exists(wpf):
            assert worker.poll() is None and time.time() - t0 < 90, "worker did not start"
            time.sleep(0.1)

        async def main():
            ok = 0
            for i in range(24):  # fresh connections: the kernel spreads them over the 3 processes
                c = InferenceClient(f"127.0.0.1:{cport}")
                for _ in range(50):
                    r = await c.call({"model": "echo", "inputs": {"x": i}, "cache": False})
                    if r.get("success"):
                        break
                    await asyncio.sleep(0.05)  # registration still propagating
                ok += bool(r.get("success"))
                c.close()
            return ok

        assert asyncio.run(main()) == 24
    finally:
        for p in (worker, coord):
            if p is not None:
                p.terminate()
                p.wait(30)
