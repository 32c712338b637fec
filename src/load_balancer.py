"""
Load balancer: picks a worker among interchangeable ones.

API from `/root/reference/src/load_balancer.py:18-348` (four strategies,
``register_worker``/``get_worker``/``update_stats``/stats, health loop).

Changes: ``active_connections`` is really tracked (use
:meth:`track` around a request, or :meth:`acquire`/:meth:`release`) so
``least_connections`` works; health-probe round trips go to a separate
``probe_latency`` and no longer pollute request latency (which skewed
``least_latency``); round-robin starts at the first worker; ``least_latency``
uses an EWMA (``latency_alpha``) so a worker that got slow is noticed, and
an unmeasured worker is tried first exactly once (cold-start exploration).
Optional ``groups`` partition workers (e.g. per shard / per role) so the
coordinator can ask for "a healthy decode worker of shard 3".

``least_latency`` for LLM workers (round 5): an end-to-end latency average
mostly measures the sizes of the requests a worker happened to get (a worker
that just served long generations looks slow), so it is not the signal. LLM
workers piggyback their engine state on every reply and health answer
(``engine_load``: running / waiting sequences, prompt tokens still to prefill,
the batch cap, KV occupancy, the EWMA decode step time and prefill time per
token — :meth:`src.engine.llm_engine.LLMEngine.load_snapshot`), and the balancer
scores each candidate by the time the NEW request is expected to take there:
the prefill backlog ahead of it, its own prompt at that worker's prefill rate,
and its output tokens at that worker's decode step time, stretched when the
running batch is over its cap. Work dispatched since the worker's last report is
added on top. Workers that report nothing (mock models) keep the latency EWMA
× (1 + active requests) score. Reference: `/root/reference/src/load_balancer.py:276-291`.
"""

from __future__ import annotations

import asyncio
import collections
import contextlib
import logging
import random
import time
import uuid
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Dict, List, Optional, Tuple

from src.rpc import RPCClient, tcp_connect_probe

logger = logging.getLogger(__name__)


UNREPORTED_MAX = 4096


class LoadBalancerStrategy(Enum):
    ROUND_ROBIN = "round_robin"
    LEAST_CONNECTIONS = "least_connections"
    RANDOM = "random"
    LEAST_LATENCY = "least_latency"


@dataclass
class WorkerStats:
    request_count: int = 0
    error_count: int = 0
    active_connections: int = 0
    total_latency: float = 0.0
    last_seen: float = field(default_factory=time.time)
    ewma_latency: Optional[float] = None
    probe_count: int = 0
    probe_latency: float = 0.0
    report: Optional[Dict[str, Any]] = None   # the worker's last engine_load (see module doc)
    # dispatches the last report does not cover yet: (sequence number, prompt tokens) in dispatch order; bounded
    # (a worker that never reports — a mock model — must not grow it without end; entries that old are covered)
    unreported: "collections.deque" = field(default_factory=lambda: collections.deque(maxlen=UNREPORTED_MAX))

    @property
    def unreported_requests(self) -> int:
        return len(self.unreported)

    @property
    def unreported_prompt_tokens(self) -> int:
        return sum(p for _, p in self.unreported)

    @property
    def avg_latency(self) -> float:
        return self.total_latency / self.request_count if self.request_count > 0 else 0.0


class LoadBalancer:
    def __init__(
        self,
        strategy: LoadBalancerStrategy = LoadBalancerStrategy.ROUND_ROBIN,
        health_check_interval: float = 5.0,
        health_check_timeout: float = 2.0,
        max_failures: int = 3,
        probe: str = "rpc",
        latency_alpha: float = 0.2,
        seed: Optional[int] = None,
        model: Optional[str] = None,
    ):
        if isinstance(strategy, str):
            strategy = LoadBalancerStrategy(strategy)
        self.strategy = strategy
        self.health_check_interval = health_check_interval
        self.health_check_timeout = health_check_timeout
        self.max_failures = max_failures
        self.probe = probe
        self.latency_alpha = latency_alpha
        self.workers: Dict[str, str] = {}
        self.worker_stats: Dict[str, WorkerStats] = {}
        self.health_checks: Dict[str, int] = {}
        self.groups: Dict[str, str] = {}
        self._rr: Dict[Optional[str], int] = {}
        self._rng = random.Random(seed)
        # the model this balancer serves (a multi-model worker's health answer carries one report per model) and
        # the token + sequence numbers of its dispatches, which workers echo in their reports (observe)
        self.model = model
        self.token = uuid.uuid4().hex[:12]
        self._seq = 0
        self._cost_ewma: Optional[Tuple[float, float]] = None
        self._running = False
        self._health_check_task: Optional[asyncio.Task] = None
        self._rpc = RPCClient(max_idle_per_host=1)
        self._strategy_fns = {
            LoadBalancerStrategy.ROUND_ROBIN: self._round_robin,
            LoadBalancerStrategy.LEAST_CONNECTIONS: self._least_connections,
            LoadBalancerStrategy.RANDOM: self._random,
            LoadBalancerStrategy.LEAST_LATENCY: self._least_latency,
        }

    async def start(self) -> None:
        if self._running:
            return
        self._running = True
        self._health_check_task = asyncio.create_task(self._health_check_loop())

    async def stop(self) -> None:
        self._running = False
        if self._health_check_task:
            self._health_check_task.cancel()
            try:
                await self._health_check_task
            except asyncio.CancelledError:
                pass
        self._rpc.close()

    # --------------------------------------------------------- membership
    def register_worker(self, worker_id: str, address: str, group: Optional[str] = None) -> None:
        self.workers[worker_id] = address
        if worker_id not in self.worker_stats:
            self.worker_stats[worker_id] = WorkerStats()
            self.health_checks[worker_id] = 0
        if group is not None:
            self.groups[worker_id] = group

    def unregister_worker(self, worker_id: str) -> bool:
        if worker_id not in self.workers:
            return False
        del self.workers[worker_id]
        self.worker_stats.pop(worker_id, None)
        self.health_checks.pop(worker_id, None)
        self.groups.pop(worker_id, None)
        return True

    def is_healthy(self, worker_id: str) -> bool:
        return worker_id in self.workers and self.health_checks.get(worker_id, 0) < self.max_failures

    # ---------------------------------------------------------- selection
    async def get_worker(self, worker_id: Optional[str] = None, group: Optional[str] = None,
                         exclude: Optional[List[str]] = None) -> Optional[Tuple[str, str]]:
        return self.pick(worker_id, group, exclude)

    def pick(self, worker_id: Optional[str] = None, group: Optional[str] = None,
             exclude: Optional[List[str]] = None, cost: Optional[Tuple[int, int]] = None) -> Optional[Tuple[str, str]]:
        """Synchronous selection (the coordinator's hot path). ``cost``: (prompt tokens, max output tokens) of the
        request, when known (least_latency uses it; see the module doc). The cost travels as an argument, never as
        balancer state, so concurrent callers on other threads / loops cannot see each other's."""
        if not self.workers:
            return None
        if worker_id:
            if self.is_healthy(worker_id):
                return worker_id, self.workers[worker_id]
            return None
        cands = [w for w in self.workers if self.is_healthy(w)
                 and (group is None or self.groups.get(w) == group)
                 and (not exclude or w not in exclude)]
        if not cands:
            return None
        if self.strategy is LoadBalancerStrategy.LEAST_LATENCY:
            wid = self._least_latency(cands, group, cost)
        else:
            wid = self._strategy_fns[self.strategy](cands, group)
        return (wid, self.workers[wid]) if wid else None

    def _round_robin(self, ids: List[str], group: Optional[str] = None) -> str:
        i = self._rr.get(group, 0) % len(ids)
        self._rr[group] = i + 1
        return ids[i]

    def _least_connections(self, ids: List[str], group: Optional[str] = None) -> str:
        least = min(self.worker_stats[w].active_connections for w in ids)
        tied = [w for w in ids if self.worker_stats[w].active_connections == least]
        return tied[0] if len(tied) == 1 else self._round_robin(tied, ("lc", group))  # type: ignore[arg-type]

    def _random(self, ids: List[str], group: Optional[str] = None) -> str:
        return self._rng.choice(ids)

    def _least_latency(self, ids: List[str], group: Optional[str] = None,
                       cost: Optional[Tuple[int, int]] = None) -> str:
        reported = [w for w in ids if self.worker_stats[w].report is not None]
        if reported:
            # engine-state scoring over the workers that report it; a silent one (just registered, not yet
            # probed) is tried once while it has nothing in flight
            silent = [w for w in ids if self.worker_stats[w].report is None
                      and self.worker_stats[w].active_connections == 0]
            if silent:
                return silent[0]
            c = cost or self._default_cost()
            return min(reported, key=lambda w: self.expected_ms(w, c))
        cold = [w for w in ids if self.worker_stats[w].ewma_latency is None
                and self.worker_stats[w].active_connections == 0]
        if cold:
            return cold[0]

        def score(w: str) -> float:  # workers without an engine report (mock models)
            s = self.worker_stats[w]
            lat = s.ewma_latency if s.ewma_latency is not None else 0.0
            return lat * (1.0 + s.active_connections)

        return min(ids, key=score)

    def _default_cost(self) -> Tuple[int, int]:
        return self._cost_ewma if self._cost_ewma is not None else (0, 1)

    def expected_ms(self, worker_id: str, cost: Tuple[int, int]) -> float:
        """Expected time (ms) for a request of ``cost`` = (prompt tokens, output tokens) on this worker, from its
        last engine report plus what was dispatched to it since."""
        s = self.worker_stats[worker_id]
        r = s.report or {}
        p, g = cost
        pf = float(r.get("prefill_us_per_token") or 0.0) / 1e3   # ms per prompt token
        step = float(r.get("step_ms") or 0.0)
        backlog = int(r.get("waiting_prompt_tokens", 0)) + s.unreported_prompt_tokens
        seqs = int(r.get("running", 0)) + int(r.get("waiting", 0)) + s.unreported_requests + 1
        cap = max(1, int(r.get("max_num_seqs") or 1))
        # the decode batch is over its cap: sequences take turns (the new one also waits for a slot)
        share = max(1.0, seqs / cap)
        # a KV pool near full preempts / delays admission
        kv = float(r.get("kv_used_frac") or 0.0)
        kv_pen = 1.0 + max(0.0, kv - 0.9) * 10.0
        return ((backlog + p) * pf + g * step * share) * kv_pen

    # ------------------------------------------------------ accounting
    def acquire(self, worker_id: str, cost: Optional[Tuple[int, int]] = None) -> int:
        """Count a dispatch; returns its sequence number (sent with the request as ``lb_seq`` next to ``lb`` =
        :attr:`token`, so that the worker's reports say which dispatches they cover)."""
        self._seq += 1
        s = self.worker_stats.get(worker_id)
        if s is not None:
            s.active_connections += 1
            s.unreported.append((self._seq, int(cost[0]) if cost else 0))
        if cost:
            c = self._cost_ewma
            self._cost_ewma = tuple(cost) if c is None else (0.9 * c[0] + 0.1 * cost[0], 0.9 * c[1] + 0.1 * cost[1])
        return self._seq

    def observe(self, worker_id: str, report: Optional[Dict[str, Any]]) -> None:
        """A worker's engine state (``engine_load`` of a reply or a health answer) replaces the last one. It covers
        the dispatches up to its ``lb_seen`` (the highest of this balancer's sequence numbers the worker had
        received when it built the report): those leave the unreported list, later ones — still on the wire or not
        yet submitted — stay counted on top (zeroing them herded bursts onto the worker that just
        replied). A report without ``lb_seen`` (another balancer's, or an older worker) covers everything."""
        if not isinstance(report, dict):
            return
        s = self.worker_stats.get(worker_id)
        if s is None:
            return
        s.report = report
        seen = report.get("lb_seen")
        if not isinstance(seen, int) or report.get("lb") not in (None, self.token):
            s.unreported.clear()
            return
        q = s.unreported
        while q and q[0][0] <= seen:
            q.popleft()

    def report_of(self, reply: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        """This balancer's model's engine report in a health answer (one per model on a multi-model worker; ADVICE
        r5: model B's balancer must not be scored with model A's queue), else None."""
        per = reply.get("engine_loads")
        if isinstance(per, dict) and self.model is not None:
            return per.get(self.model)
        if self.model is None or reply.get("models") in (None, [self.model]):
            return reply.get("engine_load")
        return None

    def release(self, worker_id: str) -> None:
        s = self.worker_stats.get(worker_id)
        if s is not None and s.active_connections > 0:
            s.active_connections -= 1

    @contextlib.asynccontextmanager
    async def track(self, worker_id: str, cost: Optional[Tuple[int, int]] = None):
        """``async with lb.track(w) as seq: ...`` — counts an active request (``seq``: its dispatch sequence
        number, see :meth:`acquire`) and records its outcome and latency."""
        seq = self.acquire(worker_id, cost)
        t0 = time.perf_counter()
        ok = False
        try:
            yield seq
            ok = True
        finally:
            self.release(worker_id)
            self.record(worker_id, ok, time.perf_counter() - t0)

    async def update_stats(self, worker_id: str, success: bool, latency: float) -> None:
        self.record(worker_id, success, latency)

    def record(self, worker_id: str, success: bool, latency: float) -> None:
        s = self.worker_stats.get(worker_id)
        if s is None:
            s = self.worker_stats[worker_id] = WorkerStats()
        s.request_count += 1
        s.total_latency += latency
        s.last_seen = time.time()
        a = self.latency_alpha
        s.ewma_latency = latency if s.ewma_latency is None else (1 - a) * s.ewma_latency + a * latency
        if success:
            self.health_checks[worker_id] = 0
        else:
            s.error_count += 1
            self.health_checks[worker_id] = self.health_checks.get(worker_id, 0) + 1

    # ------------------------------------------------------------ stats
    def get_worker_stats(self, worker_id: str) -> Optional[Dict[str, Any]]:
        s = self.worker_stats.get(worker_id)
        if s is None:
            return None
        return {
            "worker_id": worker_id,
            "address": self.workers.get(worker_id, "unknown"),
            "group": self.groups.get(worker_id),
            "request_count": s.request_count,
            "error_count": s.error_count,
            "active_connections": s.active_connections,
            "avg_latency": s.avg_latency,
            "ewma_latency": s.ewma_latency,
            "probe_count": s.probe_count,
            "avg_probe_latency": s.probe_latency / s.probe_count if s.probe_count else 0.0,
            "last_seen": s.last_seen,
            "healthy": self.is_healthy(worker_id),
            "engine_load": s.report,
        }

    def get_all_stats(self) -> Dict[str, Dict[str, Any]]:
        return {w: self.get_worker_stats(w) for w in self.workers}  # type: ignore[misc]

    def __repr__(self) -> str:
        return f"LoadBalancer(strategy={self.strategy.value}, workers={self.workers})"

    # ----------------------------------------------------------- health
    async def _health_check_loop(self) -> None:
        while self._running:
            try:
                await asyncio.sleep(self.health_check_interval)
                await self._check_all_workers()
            except asyncio.CancelledError:
                break
            except Exception as e:  # pragma: no cover
                logger.error("Error in health check loop: %s", e)

    async def _check_all_workers(self) -> None:
        if self.workers:
            await asyncio.gather(*(self._check_worker(w) for w in list(self.workers)), return_exceptions=True)

    async def _check_worker(self, worker_id: str) -> None:
        addr = self.workers.get(worker_id)
        if addr is None:
            return
        if self.probe == "tcp":
            ok, lat = await tcp_connect_probe(addr, self.health_check_timeout)
        else:
            ok, lat, reply = await self._rpc.probe(addr, self.health_check_timeout,
                                                   {"op": "health", "model": self.model, "lb": self.token})
            if ok and isinstance(reply, dict):
                self.observe(worker_id, self.report_of(reply))
        s = self.worker_stats.get(worker_id)
        if s is None:
            return
        s.probe_count += 1
        s.probe_latency += lat
        if ok:
            s.last_seen = time.time()
            self.health_checks[worker_id] = 0
        else:
            self.health_checks[worker_id] = self.health_checks.get(worker_id, 0) + 1
            if self.health_checks[worker_id] >= self.max_failures:
                logger.error("Worker %s marked as unhealthy", worker_id)
