#!/usr/bin/env python3
"""
End-to-end serving benchmark over the real RPC path:

    closed-loop clients → coordinator (TCP, framed JSON) → worker processes

* ``--mode mock`` (BASELINE config 1, CPU): 2 FakeModel workers + coordinator.
  ``--mock-latency-ms 0`` measures the plumbing ceiling (reference: 2,662 req/s
  at conc 1, ~4,251 req/s at conc 64, p50 14.8 ms — BASELINE.md);
  ``--mock-latency-ms ref`` keeps the reference's 50-150 ms sleep (reference:
  263 req/s at conc 32 on 1 worker, 294 on 2 workers).
* ``--mode llm`` (BASELINE config 2, GPU): one Llama worker per visible GPU
  (``--gpus``), requests of ``--prompt-len`` random tokens generating
  ``--gen-len`` tokens, coordinator batcher max_batch=32 / max_latency=10 ms.

Prints one JSON line per concurrency level.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from src.client import InferenceClient  # noqa: E402
from src.coordinator import Coordinator  # noqa: E402
from src.utils import percentile  # noqa: E402

REF = {  # reference measurements, Xeon 8 vCPU, same harness shape
    ("ref", 1, 1): 9.9, ("ref", 32, 1): 263.0, ("ref", 256, 1): 1615.0,
    ("ref", 1, 2): 10.0, ("ref", 32, 2): 294.0, ("ref", 256, 2): 1809.0,
    ("0", 1, 1): 2662.0, ("0", 64, 1): 4251.0, ("0", 1, 2): 3174.0, ("0", 64, 2): 4089.0,
}


def spawn_worker(wid, coord, args, gpu=None):
    fd, pf = tempfile.mkstemp()
    os.close(fd)
    os.unlink(pf)
    cmd = [sys.executable, "-m", "src.worker", "--worker-id", wid, "--host", "127.0.0.1", "--port", "0",
           "--port-file", pf, "--coordinator", coord, "--max-latency-ms", str(args.max_latency_ms)]
    env = dict(os.environ)
    if args.mode == "mock":
        cmd += ["--model", "echo", "--arch", "mock"]
        if args.mock_latency_ms != "ref":
            cmd += ["--mock-latency-ms", args.mock_latency_ms]
    else:
        cmd += ["--model", "llama", "--arch", "llama", "--preset", args.preset, "--max-batch-size", "32",
                "--max-model-len", str(max(1024, args.prompt_len + args.gen_len + 16))]
        if gpu is not None:
            env["HIP_VISIBLE_DEVICES"] = str(gpu)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=open(f"/tmp/{wid}.log", "w"))
    deadline = time.time() + 900
    while time.time() < deadline:
        if os.path.exists(pf):
            time.sleep(0.05)
            return p
        if p.poll() is not None:
            raise RuntimeError(f"worker {wid} exited; see /tmp/{wid}.log")
        time.sleep(0.1)
    p.kill()
    raise RuntimeError("worker start timeout")


class DirectClient:
    """The reference harness's shape: in-process LoadBalancer picks a worker,
    one RPC straight to it (no coordinator hop)."""

    def __init__(self, addrs, strategy):
        from src.load_balancer import LoadBalancer
        from src.rpc import RPCClient

        self.lb = LoadBalancer(strategy)
        for i, a in enumerate(addrs):
            self.lb.register_worker(f"w{i}", a)
        self.rpc = RPCClient(max_idle_per_host=1024)

    async def infer(self, model, inputs, cache=False):
        wid, addr = self.lb.pick()
        async with self.lb.track(wid):
            return await self.rpc.call(addr, {"model": model, "inputs": inputs})

    def close(self):
        self.rpc.close()


async def load(client, model, make_inputs, n, conc):
    lat = []
    sem = asyncio.Semaphore(conc)
    ok = 0

    async def one(i):
        nonlocal ok
        async with sem:
            t0 = time.perf_counter()
            r = await client.infer(model, make_inputs(i), cache=False)
            lat.append(time.perf_counter() - t0)
            ok += bool(r.get("success"))

    t0 = time.perf_counter()
    await asyncio.gather(*(one(i) for i in range(n)))
    return time.perf_counter() - t0, lat, ok


def _client_proc(caddr, n, conc, q):
    async def run():
        c = InferenceClient(caddr)
        await load(c, "echo", lambda i: {"i": i, "payload": "x" * 64}, conc, conc)  # warm connections
        t0 = time.perf_counter()
        el, lat, ok = await load(c, "echo", lambda i: {"i": i, "payload": "x" * 64}, n, conc)
        c.close()
        q.put((t0, t0 + el, lat, ok))
    asyncio.run(run())


def multi_client_load(caddr, n, conc, procs):
    """Load from several processes (one event loop cannot saturate a multi-process coordinator): each
    sends n/procs requests at conc/procs; the rate is over the union of their timed windows."""
    import multiprocessing as mp

    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_client_proc, args=(caddr, n // procs, max(1, conc // procs), q)) for _ in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(60)
    t0, t1 = min(r[0] for r in res), max(r[1] for r in res)
    return t1 - t0, [x for r in res for x in r[2]], sum(r[3] for r in res)


async def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["mock", "llm"], default="mock")
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--mock-latency-ms", default="0", help="'ref' = reference's 50-150 ms")
    ap.add_argument("--concurrency", default="1,32,64,256")
    ap.add_argument("--requests", type=int, default=2000)
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--max-latency-ms", type=float, default=10.0)
    ap.add_argument("--strategy", default="least_connections")
    ap.add_argument("--direct", action="store_true",
                    help="client-side load balancer straight to the workers (the reference harness's topology)")
    ap.add_argument("--coord-procs", type=int, default=0,
                    help="0: coordinator in this process (shares the client's event loop); N >= 1: a separate "
                         "`python -m src.coordinator --procs N` (N processes on one SO_REUSEPORT port)")
    ap.add_argument("--client-procs", type=int, default=1, help="load-generator processes (mock mode)")
    args = ap.parse_args()

    coord, cproc = None, None
    if args.coord_procs:
        fd, pf = tempfile.mkstemp()
        os.close(fd)
        os.unlink(pf)
        cproc = subprocess.Popen([sys.executable, "-m", "src.coordinator", "--listen-port", "0", "--procs",
                                  str(args.coord_procs), "--port-file", pf, "--max-latency-ms",
                                  str(args.max_latency_ms), "--strategy", args.strategy],
                                 cwd=ROOT, stdout=subprocess.DEVNULL, stderr=open("/tmp/bench_coord.log", "w"))
        for _ in range(600):
            if os.path.exists(pf):
                break
            await asyncio.sleep(0.1)
        port = int(open(pf).read())
    else:
        coord = Coordinator(port=0, max_batch_size=32, max_latency_ms=args.max_latency_ms, strategy=args.strategy,
                            health_check_interval=2.0)
        port = await coord.start()
    caddr = f"127.0.0.1:{port}"
    n_workers = args.workers if args.mode == "mock" else args.gpus
    procs = [spawn_worker(f"bw{i}", caddr, args, gpu=i if args.mode == "llm" else None) for i in range(n_workers)]
    try:
        probe = InferenceClient(caddr)
        for _ in range(600):
            if coord is not None and coord.healthy_worker_count() == n_workers:
                break
            if coord is None:  # every process of a multi-process coordinator must know every worker
                counts = []
                for _ in range(4 * max(1, args.coord_procs)):
                    c = InferenceClient(caddr)
                    counts.append((await c.call({"op": "health"})).get("workers", 0))
                    c.close()
                if min(counts) == n_workers:
                    break
            await asyncio.sleep(0.1)
        probe.close()
        if args.direct:
            client = DirectClient([w["address"] for w in (coord.router.get_worker_info(x)
                                                          for x in coord.router.workers)], args.strategy)
        else:
            client = InferenceClient(caddr)
        rng = random.Random(0)
        if args.mode == "mock":
            model = "echo"

            def make_inputs(i):
                return {"i": i, "payload": "x" * 64}
        else:
            model = "llama"

            def make_inputs(i):
                return {"prompt_token_ids": [rng.randrange(3, 120000) for _ in range(args.prompt_len)],
                        "max_tokens": args.gen_len, "ignore_eos": True}
            await load(client, model, make_inputs, 32 * n_workers, 32 * n_workers)  # warm-up
        for conc in [int(c) for c in args.concurrency.split(",")]:
            n = args.requests if args.mode == "mock" else max(conc, 3 * 32 * n_workers)
            if args.mode == "mock" and args.client_procs > 1:
                el, lat, ok = multi_client_load(caddr, n, conc, args.client_procs)
            else:
                el, lat, ok = await load(client, model, make_inputs, n, conc)
            rps = n / el
            ref = REF.get((args.mock_latency_ms, conc, n_workers)) if args.mode == "mock" else None
            print(json.dumps({
                "bench": "serve_rpc", "mode": args.mode, "workers": n_workers, "concurrency": conc,
                "topology": "client-LB->worker" if args.direct else "client->coordinator->worker",
                "coordinator_procs": args.coord_procs or "in-process", "client_procs": args.client_procs,
                "requests": n, "ok": ok, "req_per_s": round(rps, 1),
                "p50_ms": round(1e3 * percentile(lat, 50), 2), "p99_ms": round(1e3 * percentile(lat, 99), 2),
                "mock_latency_ms": args.mock_latency_ms if args.mode == "mock" else None,
                "reference_req_per_s": ref, "vs_reference": round(rps / ref, 2) if ref else None,
                "config": ({"prompt_len": args.prompt_len, "gen_len": args.gen_len, "preset": args.preset}
                           if args.mode == "llm" else {}),
            }), flush=True)
        client.close()
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        if coord is not None:
            await coord.stop()
        if cproc is not None:
            cproc.terminate()
            cproc.wait(30)


if __name__ == "__main__":
    asyncio.run(main())
