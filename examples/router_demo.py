#!/usr/bin/env python3
"""Router + LoadBalancer walkthrough: hash-affine routing, failover when a shard's
worker dies, and the four LB strategies over live mock workers.

    python examples/router_demo.py                 # scripted walkthrough
    python examples/router_demo.py --interactive   # REPL with the reference demo's commands
        (`/root/reference/examples/router_demo.py:31-42`: register / unregister / route / health /
        stats / workers / register_model / add_shard / help / exit) plus spawn / kill, which start
        and stop live in-process mock workers so health checks and failover have something real
        to probe.
"""

import argparse
import asyncio
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.config import ModelConfig  # noqa: E402
from src.load_balancer import LoadBalancer, LoadBalancerStrategy  # noqa: E402
from src.model_registry import ModelRegistry  # noqa: E402
from src.router import Router  # noqa: E402
from src.rpc import RPCClient  # noqa: E402
from src.worker import Worker  # noqa: E402


HELP = """register <worker_id> <host:port>      add a worker to the router
unregister <worker_id>                 remove it
spawn <worker_id>                      start an in-process mock worker and register it
kill <worker_id>                       stop a spawned worker (health checks will notice)
register_model <name> <version>        register a model version
add_shard <name> <version> <shard_id> <worker_id>
route <name> <version> <key>           which shard/worker serves this key
health                                 probe every worker now
stats | workers | help | exit"""


async def interactive(args):
    reg = ModelRegistry()
    router = Router(reg, health_check_interval=args.health_check_interval,
                    health_check_timeout=args.health_check_timeout,
                    max_consecutive_failures=args.max_failures, failover_enabled=not args.no_failover)
    await router.start()
    live = {}
    loop = asyncio.get_running_loop()
    print(HELP)
    while True:
        try:
            line = (await loop.run_in_executor(None, input, "router> ")).strip()
        except (EOFError, KeyboardInterrupt):
            break
        p = line.split()
        if not p:
            continue
        cmd, a = p[0], p[1:]
        try:
            if cmd in ("exit", "quit"):
                break
            elif cmd == "help":
                print(HELP)
            elif cmd == "register" and len(a) == 2:
                router.register_worker(a[0], a[1])
                print(f"registered {a[0]} at {a[1]} (health unknown until probed)")
            elif cmd == "unregister" and len(a) == 1:
                router.unregister_worker(a[0])
            elif cmd == "spawn" and len(a) == 1:
                w = Worker(a[0], host="127.0.0.1", install_signal_handlers=False)
                w.load_model(ModelConfig("echo", "", arch="mock", overrides={"latency_s": 0.001}))
                await w.start()
                live[a[0]] = w
                router.register_worker(a[0], w.address, healthy=True)
                print(f"{a[0]} listening on {w.address}")
            elif cmd == "kill" and len(a) == 1 and a[0] in live:
                await live.pop(a[0]).shutdown()
            elif cmd == "register_model" and len(a) >= 2:
                reg.register_model(a[0], a[1], a[2] if len(a) > 2 else "", {}, {})
            elif cmd == "add_shard" and len(a) == 4:
                reg.add_shard(a[0], a[1], int(a[2]), a[3])
            elif cmd == "route" and len(a) == 3:
                s = router.route_request(a[0], a[1], a[2])
                print("no healthy shard" if s is None else f"shard {s.shard_id} on {s.worker_id} "
                      f"({router.get_worker_address(s.worker_id)})")
            elif cmd == "health":
                await router._check_all_workers()
                print({w: router.get_worker_info(w)["health"] for w in router.workers})
            elif cmd == "stats":
                print(json.dumps(router.get_stats(), indent=2, default=str))
            elif cmd == "workers":
                print(json.dumps({w: router.get_worker_info(w) for w in router.workers}, indent=2, default=str))
            else:
                print("bad command; try help")
        except Exception as e:  # keep the REPL alive
            print(f"error: {e}")
    await router.stop()
    for w in live.values():
        await w.shutdown()


async def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--interactive", action="store_true")
    ap.add_argument("--health-check-interval", type=float, default=5.0)
    ap.add_argument("--health-check-timeout", type=float, default=2.0)
    ap.add_argument("--max-failures", type=int, default=3)
    ap.add_argument("--no-failover", action="store_true")
    args = ap.parse_args()
    if args.interactive:
        return await interactive(args)
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
