"""Serving paths on the MI355X: client -> coordinator -> GPU worker (llama-mini, HIP kernels,
hipGraph decode), and BASELINE config 3's worker pair — a prefill-role worker that ships the
prompt KV over the RPC socket (op kv_import) to a decode-role worker — checked token for token
against a colocated worker (same kernels, same KV bytes)."""

import asyncio

import pytest
import torch

from src.client import InferenceClient
from src.config import ModelConfig
from src.coordinator import Coordinator
from src.worker import Worker

pytestmark = pytest.mark.gpu


def gpu_cfg(name="mini", **kw):
    return ModelConfig(model_name=name, model_path="", arch="llama", preset="llama-mini", max_batch_size=8,
                       max_model_len=1024, max_num_batched_tokens=1024, num_kv_blocks=256, use_cuda_graph=True,
                       max_latency_ms=1.0, overrides=dict({"device": "cuda:0"}, **kw.pop("overrides", {})), **kw)


def test_gpu_worker_through_coordinator():
    async def main():
        w = Worker("g0", host="127.0.0.1", install_signal_handlers=False)
        assert w.load_model(gpu_cfg())
        wport = await w.start()
        coord = Coordinator(port=0, max_batch_size=8, max_latency_ms=2)
        cport = await coord.start()
        await coord.add_static_worker(f"127.0.0.1:{wport}")
        c = InferenceClient(f"127.0.0.1:{cport}")
        reqs = [{"prompt_token_ids": list(range(3 + i, 200 + 7 * i)), "max_tokens": 24, "ignore_eos": True}
                for i in range(12)]
        rs = await asyncio.wait_for(asyncio.gather(*(c.infer("mini", r) for r in reqs)), 300)
        assert all(r["success"] for r in rs), rs
        assert all(r["outputs"]["num_output_tokens"] == 24 for r in rs)
        st = (await c.call({"op": "stats"}))
        assert st["success"]
        c.close()
        await coord.stop()
        await w.shutdown()
    asyncio.run(main())


def test_gpu_streaming_matches_plain():
    """Token streaming on the GPU engine (hipGraph decode, multi-step windows deliver bursts): the
    streamed deltas concatenate to the non-streamed greedy output, through worker and coordinator."""
    async def main():
        w = Worker("gs", host="127.0.0.1", install_signal_handlers=False)
        assert w.load_model(gpu_cfg())
        wport = await w.start()
        coord = Coordinator(port=0, max_batch_size=8, max_latency_ms=2)
        cport = await coord.start()
        await coord.add_static_worker(f"127.0.0.1:{wport}")
        req = {"prompt_token_ids": list(range(5, 90)), "max_tokens": 40, "ignore_eos": True}
        cw, cc = InferenceClient(f"127.0.0.1:{wport}"), InferenceClient(f"127.0.0.1:{cport}")
        plain = await asyncio.wait_for(cw.call({"op": "infer", "model": "mini", "inputs": req}), 300)
        assert plain["success"], plain
        for client in (cw, cc):
            deltas, sizes, final = [], [], None
            async for fr in client.infer_stream("mini", req):
                if fr.get("done") is False:
                    deltas += fr["delta_token_ids"]
                    if fr["delta_token_ids"]:
                        sizes.append(len(fr["delta_token_ids"]))
                else:
                    final = fr
            assert final["success"] and deltas == plain["outputs"]["token_ids"] == final["outputs"]["token_ids"]
            # the prefill's token travels alone, whatever the engine thread's lead over the event loop
            # (round 3's driver box finished all 40 tokens before the loop's first wake-up: one frame)
            assert sizes[0] == 1 and len(sizes) >= 2, sizes
        cw.close()
        cc.close()
        await coord.stop()
        await w.shutdown()
    asyncio.run(main())


def test_gpu_disaggregated_workers_over_rpc():
    async def main():
        dec = Worker("dec", host="127.0.0.1", install_signal_handlers=False)
        assert dec.load_model(gpu_cfg(role="decode"))
        dport = await dec.start()
        pre = Worker("pre", host="127.0.0.1", install_signal_handlers=False)
        assert pre.load_model(gpu_cfg(role="prefill", overrides={"decode_worker": f"127.0.0.1:{dport}"}))
        pport = await pre.start()
        solo = Worker("solo", host="127.0.0.1", install_signal_handlers=False)
        assert solo.load_model(gpu_cfg())
        sport = await solo.start()
        cp, cs = InferenceClient(f"127.0.0.1:{pport}"), InferenceClient(f"127.0.0.1:{sport}")
        for plen in (37, 300):
            req = {"prompt_token_ids": list(range(3, 3 + plen)), "max_tokens": 20, "ignore_eos": True}
            a = await asyncio.wait_for(cp.call({"model": "mini", "inputs": req}), 300)
            b = await asyncio.wait_for(cs.call({"model": "mini", "inputs": req}), 300)
            assert a["success"] and b["success"], (a, b)
            assert a["outputs"]["disaggregated"]
            assert a["outputs"]["token_ids"] == b["outputs"]["token_ids"]
        dm = await InferenceClient(f"127.0.0.1:{dport}").call({"op": "engine_stats", "model": "mini"})
        assert dm["stats"]["prompt_tokens"] == 37 + 300     # imported, never prefilled there
        for x in (cp, cs):
            x.close()
        for w in (pre, dec, solo):
            await w.shutdown()
    asyncio.run(main())


def test_gpu_disaggregated_ipc_landing_zone(monkeypatch):
    """Prefill worker (this process) -> decode worker (a separate process on the same GPU): the
    packed prompt KV goes by device-to-device copy into the decode worker's IPC landing zone (the
    xGMI path between two GPUs of a node) and only metadata crosses the socket; tokens match a
    colocated worker."""
    import os
    import subprocess
    import sys
    import tempfile
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fd, pf = tempfile.mkstemp()
    os.close(fd)
    os.unlink(pf)
    cmd = [sys.executable, "-m", "src.worker", "--worker-id", "dec-ipc", "--host", "127.0.0.1", "--port", "0",
           "--port-file", pf, "--model", "mini", "--arch", "llama", "--preset", "llama-mini", "--role", "decode",
           "--max-batch-size", "8", "--max-model-len", "1024", "--num-kv-blocks", "256", "--max-latency-ms", "1"]
    log = tempfile.TemporaryFile()
    proc = subprocess.Popen(cmd, cwd=root, stdout=subprocess.DEVNULL, stderr=log)
    try:
        t0 = time.time()
        while not os.path.exists(pf):
            if proc.poll() is not None:
                log.seek(0)
                raise AssertionError(log.read().decode(errors="replace")[-3000:])
            assert time.time() - t0 < 240, "decode worker did not start"
            time.sleep(0.2)
        dport = int(open(pf).read())

        async def main():
            pre = Worker("pre-ipc", host="127.0.0.1", install_signal_handlers=False)
            assert pre.load_model(gpu_cfg(role="prefill", overrides={"decode_worker": f"127.0.0.1:{dport}"}))
            pport = await pre.start()
            solo = Worker("solo-ipc", host="127.0.0.1", install_signal_handlers=False)
            assert solo.load_model(gpu_cfg())
            sport = await solo.start()
            cp, cs = InferenceClient(f"127.0.0.1:{pport}"), InferenceClient(f"127.0.0.1:{sport}")
            import collections
            import random as _random

            rng = _random.Random(5)
            # different prompts one after the other: each reuses the slot the previous one gave back (first fit at
            # the zone's start) — a reused slot must never hand the decode engine a previous occupant's bytes
            for plen in (37, 300, 511, 300, 64):
                req = {"prompt_token_ids": [rng.randrange(3, 32000) for _ in range(plen)], "max_tokens": 16,
                       "ignore_eos": True}
                a = await asyncio.wait_for(cp.call({"model": "mini", "inputs": req}), 60)
                b = await asyncio.wait_for(cs.call({"model": "mini", "inputs": req}), 60)
                assert a["success"] and b["success"], (a, b)
                assert a["outputs"]["disaggregated"]
                assert a["outputs"]["token_ids"] == b["outputs"]["token_ids"]
            link = pre.models["mini"]._decode_link
            # every packet was gathered by the prefill engine straight into a slot reserved before its prompt
            # ran (one pass, no staging tensor, no second copy)
            assert link.ipc_packets == 5 and link.direct_packets == 5 and link.wire_packets == 0, \
                (link.ipc_packets, link.direct_packets, link.wire_packets)
            assert max(collections.Counter(link.slot_offsets).values()) >= 3, link.slot_offsets
            assert link.kv_path == "direct", link.stats()
            cd = InferenceClient(f"127.0.0.1:{dport}")

            async def zone():
                st = await cd.call({"op": "engine_stats", "model": "mini"})
                return st["stats"]["kv_zone"]

            async def drained():  # a slot given back by a failed sender returns once its gather finished
                for _ in range(100):
                    z = await zone()
                    if z["slots_used"] == 0 and z["reserved"] == 0:
                        return z
                    await asyncio.sleep(0.05)
                return z

            z = await zone()  # every imported slot went back behind the decode engine's scatter
            assert z["slots_used"] == 0 and z["pending_release"] == 0, z

            async def broken(*a, **k):
                raise RuntimeError("injected transfer failure")
            req = {"prompt_token_ids": list(range(9, 200)), "max_tokens": 8, "ignore_eos": True}
            # the hand-off fails after the prompt's blocks were gathered into the reserved slot: the sender
            # releases the slot behind that gather, no leak
            link._ipc.wait_ready = broken
            r = await asyncio.wait_for(cp.call({"model": "mini", "inputs": req}), 60)
            assert not r["success"]
            z = await drained()
            assert z["slots_used"] == 0 and z["reserved"] == 0, z
            del link._ipc.wait_ready
            # the staged path (kv_direct off: packed copy into the slot after kv_reserve) with a failing copy
            pre.models["mini"].kv_direct = False
            try:
                link._ipc.write_async = broken
                r = await asyncio.wait_for(cp.call({"model": "mini", "inputs": req}), 60)
                assert not r["success"]
                z = await drained()
                assert z["slots_used"] == 0 and z["reserved"] == 0, z
                del link._ipc.write_async
                r = await asyncio.wait_for(cp.call({"model": "mini", "inputs": req}), 60)
                assert r["success"] and r["outputs"]["disaggregated"]
            finally:
                pre.models["mini"].kv_direct = True
            r = await asyncio.wait_for(cp.call({"model": "mini", "inputs": req}), 60)
            assert r["success"] and r["outputs"]["disaggregated"]
            assert link.wire_packets == 0 and link.direct_packets == 6, (link.wire_packets, link.direct_packets)
            cd.close()
            for x in (cp, cs):
                x.close()
            for w in (pre, solo):
                await w.shutdown()
        asyncio.run(main())
    except BaseException:
        log.seek(0)
        print("decode worker log:\n" + log.read().decode(errors="replace")[-4000:], flush=True)
        raise
    finally:
        proc.terminate()
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            proc.kill()



def test_lb_serving_rehearsal_one_gpu(capsys):
    """Config 5's balancer on real GPU worker processes: three llama-mini workers (src.worker,
    RPC) share cuda:0 behind the coordinator, one with a 2-sequence batch cap; least_latency (scoring each request on
    the workers' engine reports) and round_robin both serve the mixed, prefix-sharing workload completely, and
    least_latency sends the slow worker a smaller share of the requests than round robin's third."""
    import importlib.util
    import json
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench", "lb_serving_bench.py")
    spec = importlib.util.spec_from_file_location("lb_serving_bench", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rc = mod.main(["--preset", "llama-mini", "--device", "cuda:0", "--workers", "3", "--slow", "1", "--batch", "16",
                   "--slow-batch", "2", "--kv-blocks", "256", "--requests", "96", "--concurrency", "24",
                   "--prompt-min", "64", "--prompt-max", "512", "--gen", "16,32,64"])
    assert rc == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.splitlines() if x.startswith("{")]
    runs = {x["strategy"]: x for x in lines if "strategy" in x}
    for r in runs.values():
        assert r["requests"] == 96 and r["error_count"] == 0, r
    summ = lines[-1]
    assert summ["slow_share_ll"] < summ["slow_share_rr"], summ
