"""
Router: request-key → shard placement with health tracking and failover.

API from `/root/reference/src/router.py:27-358`. Placement asks the registry
for the key's shard (rendezvous hashing, see :mod:`src.model_registry`); if
that shard's worker is unknown or unhealthy and failover is on, the key is
re-placed deterministically among the healthy shards
(`router.py:186-221`). On MI355X a shard is a placement unit — a DP replica on
one GPU, a TP group, or a prefill/decode pair — so "failover" moves a session
to another replica; a TP group fails as a unit because its shard has one
entry worker (rank 0).

Changes vs the reference:

* ``register_worker(..., healthy=True)`` marks a worker HEALTHY when it joins
  through a successful registration handshake, instead of leaving it UNKNOWN
  (and unroutable) until the first probe ``health_check_interval`` later;
* probes are real ``{"op":"health"}`` RPCs (``probe="rpc"``, default) or the
  reference's bare TCP connect (``probe="tcp"``);
* ``load_aware=True`` breaks failover ties by ``ModelShard.load`` (the
  "load-aware routing (optional)" the reference advertises but never reads).
"""

from __future__ import annotations

import asyncio
import logging
import time
from dataclasses import dataclass, field
from enum import Enum, auto
from typing import Any, Dict, List, Optional

from src.model_registry import ModelRegistry, ModelShard, ModelStatus, rendezvous_score
from src.rpc import RPCClient, tcp_connect_probe

logger = logging.getLogger(__name__)


class WorkerHealth(Enum):
    HEALTHY = auto()
    UNHEALTHY = auto()
    UNKNOWN = auto()


@dataclass
class WorkerInfo:
    worker_id: str
    address: str
    health: WorkerHealth = WorkerHealth.UNKNOWN
    last_health_check: float = 0.0
    consecutive_failures: int = 0
    last_success: float = 0.0
    metadata: Dict[str, Any] = field(default_factory=dict)


class Router:
    def __init__(
        self,
        registry: ModelRegistry,
        health_check_interval: float = 5.0,
        health_check_timeout: float = 2.0,
        max_consecutive_failures: int = 3,
        failover_enabled: bool = True,
        probe: str = "rpc",
        load_aware: bool = False,
    ):
        self.registry = registry
        self.health_check_interval = health_check_interval
        self.health_check_timeout = health_check_timeout
        self.max_consecutive_failures = max_consecutive_failures
        self.failover_enabled = failover_enabled
        self.probe = probe
        self.load_aware = load_aware
        self.workers: Dict[str, WorkerInfo] = {}
        self._health_check_task: Optional[asyncio.Task] = None
        self._running = False
        self._rpc = RPCClient(max_idle_per_host=1)
        self.routed = 0
        self.failovers = 0
        self.route_failures = 0

    async def start(self) -> None:
        if self._running:
            logger.warning("Router is already running")
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
    def register_worker(self, worker_id: str, address: str, metadata: Optional[Dict[str, Any]] = None,
                        healthy: bool = False) -> None:
        if worker_id in self.workers:
            logger.info("Worker %s re-registered", worker_id)
        now = time.time()
        self.workers[worker_id] = WorkerInfo(
            worker_id=worker_id,
            address=address,
            health=WorkerHealth.HEALTHY if healthy else WorkerHealth.UNKNOWN,
            last_success=now if healthy else 0.0,
            metadata=metadata or {},
        )

    def unregister_worker(self, worker_id: str) -> None:
        self.workers.pop(worker_id, None)

    # ------------------------------------------------------------ routing
    def route_request(self, model_name: str, version: str, request_key: str,
                      prefer_healthy: bool = True) -> Optional[ModelShard]:
        shard = self.registry.get_shard_for_key(model_name, version, request_key)
        if shard is None:
            self.route_failures += 1
            return None
        info = self.workers.get(shard.worker_id)
        usable = info is not None and shard.status == ModelStatus.READY and (
            not prefer_healthy or info.health == WorkerHealth.HEALTHY)
        if usable:
            self.routed += 1
            return shard
        if not self.failover_enabled:
            self.route_failures += 1
            return None
        alt = self._find_alternative_shard(model_name, version, request_key)
        if alt is None:
            self.route_failures += 1
        else:
            self.routed += 1
            self.failovers += 1
        return alt

    def healthy_shards(self, model_name: str, version: str) -> List[ModelShard]:
        mv = self.registry.get_model_version(model_name, version)
        if mv is None:
            return []
        out = []
        for s in mv.shards:
            w = self.workers.get(s.worker_id)
            if w is not None and w.health == WorkerHealth.HEALTHY and s.status == ModelStatus.READY:
                out.append(s)
        return out

    def _find_alternative_shard(self, model_name: str, version: str, request_key: str) -> Optional[ModelShard]:
        healthy = self.healthy_shards(model_name, version)
        if not healthy:
            logger.error("No healthy shards available for %s:%s", model_name, version)
            return None
        if self.load_aware:
            least = min(s.load for s in healthy)
            healthy = [s for s in healthy if s.load <= least + 0.25]
        # Deterministic per key among the survivors (same key → same backup).
        return max(healthy, key=lambda s: rendezvous_score(request_key, s.shard_id))

    # ------------------------------------------------------------- health
    def mark_worker_success(self, worker_id: str) -> None:
        w = self.workers.get(worker_id)
        if w is None:
            return
        w.last_success = time.time()
        w.consecutive_failures = 0
        if w.health != WorkerHealth.HEALTHY:
            w.health = WorkerHealth.HEALTHY
            logger.info("Worker %s marked healthy", worker_id)

    def mark_worker_failure(self, worker_id: str) -> None:
        w = self.workers.get(worker_id)
        if w is None:
            return
        w.consecutive_failures += 1
        if w.consecutive_failures >= self.max_consecutive_failures and w.health != WorkerHealth.UNHEALTHY:
            w.health = WorkerHealth.UNHEALTHY
            logger.warning("Worker %s marked unhealthy (%d consecutive failures)", worker_id,
                           w.consecutive_failures)

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
            await asyncio.gather(*(self._check_worker_health(w) for w in list(self.workers)),
                                 return_exceptions=True)

    async def _check_worker_health(self, worker_id: str) -> None:
        w = self.workers.get(worker_id)
        if w is None:
            return
        if self.probe == "tcp":
            ok, _ = await tcp_connect_probe(w.address, self.health_check_timeout)
        else:
            ok, _, reply = await self._rpc.probe(w.address, self.health_check_timeout)
            if ok and isinstance(reply, dict) and "load" in reply:
                w.metadata["load"] = reply["load"]
        w.last_health_check = time.time()
        if ok:
            self.mark_worker_success(worker_id)
        else:
            self.mark_worker_failure(worker_id)

    # ------------------------------------------------------------ queries
    def get_worker_address(self, worker_id: str) -> Optional[str]:
        w = self.workers.get(worker_id)
        return w.address if w else None

    def get_healthy_workers(self) -> List[str]:
        return [k for k, w in self.workers.items() if w.health == WorkerHealth.HEALTHY]

    def get_unhealthy_workers(self) -> List[str]:
        return [k for k, w in self.workers.items() if w.health == WorkerHealth.UNHEALTHY]

    def get_stats(self) -> Dict[str, Any]:
        total = len(self.workers)
        healthy = len(self.get_healthy_workers())
        unhealthy = len(self.get_unhealthy_workers())
        return {
            "total_workers": total,
            "healthy_workers": healthy,
            "unhealthy_workers": unhealthy,
            "unknown_workers": total - healthy - unhealthy,
            "failover_enabled": self.failover_enabled,
            "health_check_interval": self.health_check_interval,
            "routed": self.routed,
            "failovers": self.failovers,
            "route_failures": self.route_failures,
        }

    def get_worker_info(self, worker_id: str) -> Optional[Dict[str, Any]]:
        w = self.workers.get(worker_id)
        if w is None:
            return None
        return {
            "worker_id": w.worker_id,
            "address": w.address,
            "health": w.health.name,
            "consecutive_failures": w.consecutive_failures,
            "last_health_check": w.last_health_check,
            "last_success": w.last_success,
            "metadata": w.metadata,
        }
