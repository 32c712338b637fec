"""Router + LoadBalancer: strategies, health, failover, accounting."""

import asyncio

import pytest

from src.load_balancer import LoadBalancer, LoadBalancerStrategy
from src.model_registry import ModelRegistry
from src.router import Router, WorkerHealth


def _registry(n=3):
    reg = ModelRegistry()
    reg.register_model("m", "1", "/p", {}, {})
    for i in range(n):
        reg.add_shard("m", "1", i, f"w{i}")
    return reg


def test_route_and_failover():
    reg = _registry()
    r = Router(reg, max_consecutive_failures=2)
    for i in range(3):
        r.register_worker(f"w{i}", f"127.0.0.1:{1000 + i}", healthy=True)
    s = r.route_request("m", "1", "user-7")
    assert s is not None and r.route_request("m", "1", "user-7").shard_id == s.shard_id
    r.mark_worker_failure(s.worker_id)
    r.mark_worker_failure(s.worker_id)
    assert r.workers[s.worker_id].health == WorkerHealth.UNHEALTHY
    alt = r.route_request("m", "1", "user-7")
    assert alt.shard_id != s.shard_id
    assert r.route_request("m", "1", "user-7").shard_id == alt.shard_id  # deterministic backup
    r.mark_worker_success(s.worker_id)
    assert r.route_request("m", "1", "user-7").shard_id == s.shard_id
    r2 = Router(reg, failover_enabled=False)
    assert r2.route_request("m", "1", "k") is None    # workers not registered
    assert r.get_stats()["failovers"] >= 1


def test_unknown_until_probed_unless_handshake():
    reg = _registry(1)
    r = Router(reg)
    r.register_worker("w0", "127.0.0.1:1")
    assert r.route_request("m", "1", "k") is None
    r.register_worker("w0", "127.0.0.1:1", healthy=True)
    assert r.route_request("m", "1", "k").worker_id == "w0"


def test_health_probe_marks_dead_worker():
    async def main():
        reg = _registry(1)
        r = Router(reg, health_check_interval=0.01, health_check_timeout=0.2, max_consecutive_failures=2)
        r.register_worker("w0", "127.0.0.1:1", healthy=True)     # nothing listens on port 1
        await r.start()
        await asyncio.sleep(0.3)
        await r.stop()
        assert r.workers["w0"].health == WorkerHealth.UNHEALTHY
    asyncio.run(main())


def test_lb_round_robin_and_groups():
    lb = LoadBalancer(LoadBalancerStrategy.ROUND_ROBIN)
    for i in range(3):
        lb.register_worker(f"w{i}", f"a:{i}", group="g0" if i < 2 else "g1")
    picks = [lb.pick()[0] for _ in range(6)]
    assert picks == ["w0", "w1", "w2"] * 2
    assert {lb.pick(group="g0")[0] for _ in range(4)} == {"w0", "w1"}
    assert lb.pick(group="g1")[0] == "w2"
    assert lb.pick(worker_id="w1") == ("w1", "a:1")
    assert lb.pick(exclude=["w0", "w1"])[0] == "w2"


def test_lb_least_connections_tracks_active():
    async def main():
        lb = LoadBalancer(LoadBalancerStrategy.LEAST_CONNECTIONS)
        lb.register_worker("a", "x:1")
        lb.register_worker("b", "x:2")
        counts = {"a": 0, "b": 0}
        gate = asyncio.Event()

        async def req():
            w, _ = lb.pick()
            counts[w] += 1
            async with lb.track(w):
                await gate.wait()

        ts = [asyncio.create_task(req()) for _ in range(10)]
        await asyncio.sleep(0.01)
        gate.set()
        await asyncio.gather(*ts)
        assert counts == {"a": 5, "b": 5}
        assert lb.worker_stats["a"].active_connections == 0
    asyncio.run(main())


def test_lb_least_latency_prefers_fast_and_explores_cold():
    lb = LoadBalancer(LoadBalancerStrategy.LEAST_LATENCY)
    lb.register_worker("slow", "x:1")
    lb.register_worker("fast", "x:2")
    lb.record("slow", True, 0.5)
    assert lb.pick()[0] == "fast"           # cold worker explored first
    lb.record("fast", True, 0.05)
    assert all(lb.pick()[0] == "fast" for _ in range(5))
    for _ in range(20):
        lb.record("fast", True, 2.0)        # fast got slow: EWMA notices
    assert lb.pick()[0] == "slow"


def test_lb_failures_make_unhealthy():
    lb = LoadBalancer(max_failures=2)
    lb.register_worker("a", "x:1")
    lb.register_worker("b", "x:2")
    lb.record("a", False, 0.1)
    lb.record("a", False, 0.1)
    assert not lb.is_healthy("a")
    assert {lb.pick()[0] for _ in range(4)} == {"b"}
    assert lb.pick(worker_id="a") is None
    lb.record("a", True, 0.1)
    assert lb.is_healthy("a")
    assert lb.unregister_worker("a") and not lb.unregister_worker("a")
    st = lb.get_worker_stats("b")
    assert st["healthy"] and st["request_count"] == 0


def test_lb_random_seeded():
    lb = LoadBalancer("random", seed=1)
    for i in range(4):
        lb.register_worker(f"w{i}", f"x:{i}")
    assert len({lb.pick()[0] for _ in range(100)}) == 4
