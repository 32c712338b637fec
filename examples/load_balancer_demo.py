#!/usr/bin/env python3
"""Load-balancer demo (the reference's `examples/load_balancer_demo.py:27-238`, re-done so
requests really travel over RPC to live workers).

For each strategy: start N in-process mock workers (worker-1 is 5x slower than
the rest), send `--requests` requests with `--concurrency` in flight through the
LoadBalancer (`track()` counts in-flight requests, so least_connections sees
real load; the measured RPC latency feeds least_latency), and for round_robin
kill worker-2 halfway through to show failover: the failed RPC is recorded,
the worker is taken out of rotation, and the request is retried elsewhere.

    python examples/load_balancer_demo.py --workers 3 --requests 60
"""

import argparse
import asyncio
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.config import ModelConfig  # noqa: E402
from src.load_balancer import LoadBalancer, LoadBalancerStrategy  # noqa: E402
from src.rpc import RPCClient  # noqa: E402
from src.worker import Worker  # noqa: E402


async def start_workers(n: int, base_latency_s: float):
    workers = []
    for i in range(n):
        w = Worker(f"worker-{i + 1}", host="127.0.0.1", install_signal_handlers=False)
        lat = base_latency_s * (5 if i == 0 else 1)
        w.load_model(ModelConfig("test-model", f"models/worker-{i + 1}", batch_size=8, max_batch_size=32,
                                 input_schema={"input": "string"}, output_schema={"output": "string"},
                                 arch="mock", overrides={"latency_s": lat}))
        await w.start()
        workers.append(w)
    return workers


async def run_strategy(strategy: LoadBalancerStrategy, args) -> None:
    print(f"\n{'=' * 60}\n{strategy.value.upper()}\n{'=' * 60}")
    workers = await start_workers(args.workers, args.latency_ms / 1e3)
    lb = LoadBalancer(strategy, health_check_interval=0.2, max_failures=1, seed=0)
    for w in workers:
        lb.register_worker(w.worker_id, w.address)
    await lb.start()
    rpc = RPCClient()
    counts = collections.Counter()
    failures = 0
    sem = asyncio.Semaphore(args.concurrency)
    kill_at = args.requests // 2 if strategy == LoadBalancerStrategy.ROUND_ROBIN and len(workers) > 1 else -1

    async def one(i: int):
        nonlocal failures
        async with sem:
            if i == kill_at:
                print(f"  request {i}: stopping {workers[1].worker_id} (simulated failure)")
                await workers[1].shutdown()
            for _attempt in range(3):
                picked = lb.pick()
                if picked is None:
                    print("  no healthy workers")
                    return
                wid, addr = picked
                lb.acquire(wid)  # in-flight count for least_connections
                t0 = time.perf_counter()
                try:
                    r = await rpc.call(addr, {"model": "test-model", "inputs": {"input": f"req-{i}"}},
                                       timeout=5.0)
                    ok = bool(r.get("success"))
                except (OSError, asyncio.TimeoutError, ConnectionError):
                    ok = False
                finally:
                    lb.release(wid)
                lb.record(wid, ok, time.perf_counter() - t0)  # failure → out of rotation (max_failures=1)
                if ok:
                    counts[wid] += 1
                    return
                failures += 1

    t0 = time.perf_counter()
    await asyncio.gather(*(one(i) for i in range(args.requests)))
    el = time.perf_counter() - t0
    print(f"  {args.requests} requests in {el:.2f} s ({args.requests / el:.1f} req/s), "
          f"{failures} failed attempts retried")
    print("  distribution:", dict(sorted(counts.items())))
    for wid, st in sorted(lb.get_all_stats().items()):
        if st:
            print(f"  {wid}: requests={st['request_count']} errors={st['error_count']} "
                  f"avg_latency={st['avg_latency'] * 1e3:.1f} ms healthy={st['healthy']}")
    await lb.stop()
    rpc.close()
    for w in workers:
        if w.server is not None:
            await w.shutdown()


async def main():
    ap = argparse.ArgumentParser(description="Load Balancer Demo")
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--requests", type=int, default=60)
    ap.add_argument("--concurrency", type=int, default=6)
    ap.add_argument("--latency-ms", type=float, default=10.0, help="base mock latency (worker-1 is 5x)")
    ap.add_argument("--strategy", choices=[s.value for s in LoadBalancerStrategy], default=None)
    args = ap.parse_args()
    strategies = [LoadBalancerStrategy(args.strategy)] if args.strategy else list(LoadBalancerStrategy)
    for s in strategies:
        await run_strategy(s, args)


if __name__ == "__main__":
    asyncio.run(main())
