#!/usr/bin/env python3
"""Router + LoadBalancer walkthrough (scripted; the reference's router and
load-balancer demos, re-done): hash-affine routing, failover when a shard's
worker dies, and the four LB strategies over live mock workers."""

import asyncio
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.config import ModelConfig  # noqa: E402
from src.load_balancer import LoadBalancer, LoadBalancerStrategy  # noqa: E402
from src.model_registry import ModelRegistry  # noqa: E402
from src.router import Router  # noqa: E402
from src.rpc import RPCClient  # noqa: E402
from src.worker import Worker  # noqa: E402


async def main():
    workers = []
    for i in range(3):
        w = Worker(f"w{i}", host="127.0.0.1", install_signal_handlers=False)
        w.load_model(ModelConfig("echo", "", arch="mock", overrides={"latency_s": 0.002 * (i + 1)}))
        await w.start()
        workers.append(w)
    reg = ModelRegistry()
    reg.register_model("echo", "1", "", {}, {})
    router = Router(reg, health_check_interval=0.2, max_consecutive_failures=1)
    for i, w in enumerate(workers):
        reg.add_shard("echo", "1", i, w.worker_id)
        router.register_worker(w.worker_id, w.address, healthy=True)
    await router.start()
    keys = [f"user-{i}" for i in range(12)]
    print("placement:", {k: router.route_request("echo", "1", k).worker_id for k in keys})
    await workers[1].shutdown()
    await asyncio.sleep(0.5)
    print("after w1 died:", {k: router.route_request("echo", "1", k).worker_id for k in keys})
    print("router stats:", router.get_stats())
    await router.stop()

    rpc = RPCClient()
    live = [w for w in workers if w.server is not None]
    for strat in LoadBalancerStrategy:
        lb = LoadBalancer(strat, seed=0)
        for w in live:
            lb.register_worker(w.worker_id, w.address)
        counts = collections.Counter()
        for i in range(40):
            wid, addr = lb.pick()
            async with lb.track(wid):
                await rpc.call(addr, {"model": "echo", "inputs": i})
            counts[wid] += 1
        print(f"{strat.value:>18}: {dict(counts)}  avg latency "
              f"{ {w: round(1e3 * lb.worker_stats[w].avg_latency, 1) for w in lb.workers} } ms")
    rpc.close()
    for w in live:
        await w.shutdown()


if __name__ == "__main__":
    asyncio.run(main())
