"""
Coordinator: the serving front door.

The reference documents it (`/root/reference/README.md:27,56-60,109`,
`docs/router_vs_load_balancer.md:41-57`) but never ships it. Request flow:

    client ──framed JSON──▶ Coordinator.handle_request
       ├─ validate {"model", "inputs", ["version"], ["request_key"], ["cache"]}
       ├─ response cache (KVCache) hit → reply            (README.md:57-60)
       ├─ shard  = Router.route_request(model, version, request_key)   (hash affinity + failover)
       ├─ fut    = Batcher.add_request(model, "version#shard", inputs)  (max_batch / max_latency admission)
       │     batch_callback → LoadBalancer.pick(group=shard) → RPC to the worker
       │       "batch"  dispatch: one infer_batch RPC per flushed batch (coalesced; mock models)
       │       "stream" dispatch: one infer RPC per request, all in flight at once; the worker's
       │                 continuous-batching engine re-batches them per token step (LLMs)
       │     failure → LB.record(failure) + Router.mark_worker_failure → retry on another
       │               worker of the shard, then on another healthy shard (README.md:60 retries)
       ├─ await fut → cache.set → reply, or ``op:"submit"`` returns a request_id to poll
       └─ Tracer marks every stage (TTFT/TPOT come back in the LLM outputs)

Workers join through ``{"op":"register"}`` (the handshake of README.md:85) or
are listed statically (``--worker host:port``, or ``examples/demo_config.yaml``).
"""

from __future__ import annotations

import asyncio
import contextlib
import hashlib
import json
import logging
import os
import time
from typing import Any, Dict, List, Optional, Tuple

if __package__ in (None, ""):  # `python src/coordinator.py`
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.batcher import Batcher  # noqa: E402
from src.config import DeploymentConfig  # noqa: E402
from src.kvstore import KVCache  # noqa: E402
from src.load_balancer import LoadBalancer, LoadBalancerStrategy  # noqa: E402
from src.model_registry import ModelRegistry, rendezvous_score  # noqa: E402
from src.preproc import request_cost  # noqa: E402
from src.router import Router, WorkerHealth  # noqa: E402
from src.rpc import RPCClient, RPCError  # noqa: E402
from src.utils import (  # noqa: E402
    CODEC_MSGPACK,
    GLOBAL_TRACER,
    new_request_id,
    setup_logging,
)
from src.utils.frameserver import start_frame_server  # noqa: E402

logger = logging.getLogger(__name__)

DEFAULT_VERSION = "1.0"


class Coordinator:
    def __init__(
        self,
        host: str = "127.0.0.1",
        port: int = 9000,
        strategy: str = "round_robin",
        max_batch_size: int = 32,
        max_latency_ms: float = 10.0,
        batch_idle_flush_ms: Optional[float] = 1.0,
        cache_size: int = 10000,
        cache_policy: str = "lru",
        cache_ttl_s: Optional[float] = None,
        max_retries: int = 2,
        request_timeout_s: float = 600.0,
        health_check_interval: float = 5.0,
        dispatch: Optional[str] = None,
        reuse_port: bool = False,
    ):
        self.host, self.port = host, port
        # several coordinator processes may share one listening port (SO_REUSEPORT: the kernel spreads
        # connections over them); they forward worker (un)registrations to each other (peer_addrs)
        self.reuse_port = reuse_port
        self.peer_addrs: List[str] = []
        self.peer_server: Optional[asyncio.AbstractServer] = None
        self.strategy = LoadBalancerStrategy(strategy)
        self.max_retries = max_retries
        self.request_timeout_s = request_timeout_s
        self.health_check_interval = health_check_interval
        self.dispatch_override = dispatch
        self.registry = ModelRegistry()
        self.router = Router(self.registry, health_check_interval=health_check_interval)
        self.lbs: Dict[str, LoadBalancer] = {}
        self.cache = KVCache(max_size=cache_size, eviction_policy=cache_policy, default_ttl=cache_ttl_s)
        # eager_when_idle: an idle shard gets a request immediately; max_latency only
        # applies while a previous batch for that shard is still in flight.
        self.batcher = Batcher(max_batch_size=max_batch_size, max_latency_ms=max_latency_ms,
                               batch_callback=self._batch_callback, eager_when_idle=True,
                               idle_flush_ms=batch_idle_flush_ms)
        # coordinator -> worker frames in msgpack (C codec: ~3x cheaper than json per hop); clients keep JSON
        self.rpc = RPCClient(max_idle_per_host=512, codec=CODEC_MSGPACK)
        self.tracer = GLOBAL_TRACER
        self.server: Optional[asyncio.AbstractServer] = None
        self._pending: Dict[str, asyncio.Task] = {}
        self._results: KVCache = KVCache(max_size=100000, default_ttl=3600)
        self._model_arch: Dict[str, str] = {}
        self._shard_ids: Dict[str, int] = {}
        self.stats = {"requests": 0, "errors": 0, "cache_hits": 0, "retries": 0, "registrations": 0}

    @classmethod
    def from_config(cls, cfg: DeploymentConfig) -> "Coordinator":
        return cls(host=cfg.listen_host, port=cfg.listen_port, strategy=cfg.strategy,
                   max_batch_size=cfg.batch_max_size, max_latency_ms=cfg.batch_max_latency_ms,
                   batch_idle_flush_ms=cfg.batch_idle_flush_ms, cache_size=cfg.cache_size,
                   cache_policy=cfg.cache_policy, cache_ttl_s=cfg.cache_ttl_s,
                   max_retries=cfg.max_retries, request_timeout_s=cfg.request_timeout_s,
                   health_check_interval=cfg.health_check_interval)

    # ----------------------------------------------------------- lifecycle
    async def start(self) -> int:
        await self.batcher.start()
        await self.router.start()
        for lb in self.lbs.values():
            await lb.start()
        # backlog: a burst of >100 new client connections must not hit SYN retransmits (1 s stalls)
        # protocol-level framing (src/utils/frameserver.py): no reader task per request on the front door
        self.server = await start_frame_server(self.handle_message, self.host, self.port, backlog=4096,
                                               reuse_port=self.reuse_port or None)
        self.port = self.server.sockets[0].getsockname()[1]
        logger.info("Coordinator listening on %s:%d", self.host, self.port)
        return self.port

    async def start_peer_server(self) -> str:
        """A private listener on which sibling coordinator processes reach THIS process (forwarded
        registrations); returns its address."""
        self.peer_server = await start_frame_server(self.handle_message, self.host, 0)
        return f"{self.host}:{self.peer_server.sockets[0].getsockname()[1]}"

    async def _forward(self, msg: Dict[str, Any]) -> None:
        fwd = dict(msg, _fwd=True)
        for a in self.peer_addrs:
            try:
                await self.rpc.call(a, fwd, timeout=10.0)
            except Exception as e:  # a sibling that is down re-learns membership from health checks
                logger.warning("forwarding %s to sibling %s failed: %s", msg.get("op"), a, e)

    async def stop(self) -> None:
        if self.peer_server:
            self.peer_server.close()
        if self.server:
            self.server.close()
            with contextlib.suppress(Exception):
                await asyncio.wait_for(self.server.wait_closed(), 2.0)
        await self.batcher.stop()
        await self.router.stop()
        for lb in self.lbs.values():
            await lb.stop()
        for t in self._pending.values():
            t.cancel()
        self.rpc.close()

    # -------------------------------------------------------- membership
    def _lb(self, model: str, version: str) -> LoadBalancer:
        key = f"{model}:{version}"
        lb = self.lbs.get(key)
        if lb is None:
            lb = self.lbs[key] = LoadBalancer(strategy=self.strategy,
                                              health_check_interval=self.health_check_interval, model=model)
            if self.server is not None:
                asyncio.get_event_loop().create_task(lb.start())
        return lb

    def register_worker(self, worker_id: str, address: str, models: Dict[str, Dict[str, Any]],
                        metadata: Optional[Dict[str, Any]] = None, healthy: bool = True) -> None:
        """Add a worker and the models it serves. ``metadata["shard_id"]``
        puts it into an existing shard (replica); otherwise it forms a new one."""
        metadata = dict(metadata or {})
        self.router.register_worker(worker_id, address, metadata, healthy=healthy)
        for name, mcfg in models.items():
            mcfg = mcfg or {}
            version = str(mcfg.get("overrides", {}).get("version", mcfg.get("version", DEFAULT_VERSION)))
            if self.registry.get_model_version(name, version) is None:
                self.registry.register_model(
                    name, version, mcfg.get("model_path", ""), mcfg.get("input_schema") or {},
                    mcfg.get("output_schema") or {}, batch_size=mcfg.get("batch_size", 1),
                    max_batch_size=mcfg.get("max_batch_size", 32),
                    metadata={"arch": mcfg.get("arch", "mock"), "preset": mcfg.get("preset")})
            self._model_arch[name] = mcfg.get("arch", "mock")
            shard_id = metadata.get("shard_id")
            if shard_id is None:
                key = f"{name}:{version}"
                shard_id = self._shard_ids.get(key, 0)
                self._shard_ids[key] = shard_id + 1
            self.registry.add_shard(name, version, int(shard_id), worker_id, metadata)
            self._lb(name, version).register_worker(worker_id, address, group=str(shard_id))
        self.stats["registrations"] += 1

    def unregister_worker(self, worker_id: str) -> None:
        self.router.unregister_worker(worker_id)
        for lb in self.lbs.values():
            lb.unregister_worker(worker_id)

    async def add_static_worker(self, address: str, attempts: int = 100) -> bool:
        """Discover a worker listed on the command line via its health RPC."""
        for _ in range(attempts):
            ok, _, rep = await self.rpc.probe(address, 2.0)
            if ok and rep:
                wid = rep.get("worker_id", address)
                archs = rep.get("archs", {})
                self.register_worker(wid, address, {m: {"arch": archs.get(m, "mock")} for m in rep.get("models", [])})
                return True
            await asyncio.sleep(0.2)
        logger.error("static worker %s never answered", address)
        return False

    # --------------------------------------------------------------- serve
    async def handle_message(self, msg: Any, emit=None) -> Dict[str, Any]:
        if not isinstance(msg, dict):
            return {"error": "Request must be a JSON object", "success": False}
        op = msg.get("op", "infer")
        if op == "infer":
            inp = msg.get("inputs")
            if emit is not None and isinstance(inp, dict) and inp.get("stream"):
                return await self.handle_stream(msg, emit)
            return await self.handle_request(msg)
        if op == "submit":
            rid = msg.get("request_id") or new_request_id()
            msg = dict(msg, request_id=rid)
            task = asyncio.create_task(self.handle_request(msg))
            self._pending[rid] = task
            task.add_done_callback(lambda t, r=rid: self._finish_async(r, t))
            return {"success": True, "request_id": rid, "status": "pending"}
        if op == "result":
            rid = msg.get("request_id")
            res = self._results.get(rid)
            if res is not None:
                return res
            if rid in self._pending:
                return {"success": True, "request_id": rid, "status": "pending"}
            return {"error": f"unknown request_id {rid!r}", "success": False}
        if op == "register":
            self.register_worker(msg["worker_id"], msg["address"], msg.get("models", {}), msg.get("metadata"))
            if self.peer_addrs and not msg.get("_fwd"):
                await self._forward(msg)
            return {"success": True}
        if op == "unregister":
            self.unregister_worker(msg["worker_id"])
            if self.peer_addrs and not msg.get("_fwd"):
                await self._forward(msg)
            return {"success": True}
        if op == "health":
            return {"success": True, "role": "coordinator", "workers": len(self.router.workers)}
        if op == "stats":
            return {"success": True, "stats": await self.get_stats()}
        if op == "models":
            return {"success": True, "models": {m: self.registry.list_versions(m) for m in self.registry.list_models()}}
        return {"error": f"unknown op {op!r}", "success": False}

    def _finish_async(self, rid: str, task: asyncio.Task) -> None:
        self._pending.pop(rid, None)
        if task.cancelled():
            return
        exc = task.exception()
        res = {"error": str(exc), "success": False} if exc else task.result()
        res = dict(res, request_id=rid, status="done")
        self._results.set(rid, res)

    @staticmethod
    def _cache_key(model: str, version: str, inputs: Any) -> Optional[str]:
        try:
            blob = json.dumps([model, version, inputs], sort_keys=True, separators=(",", ":"))
        except (TypeError, ValueError):
            return None
        return hashlib.blake2b(blob.encode(), digest_size=16).hexdigest()

    def _cacheable(self, model: str, msg: Dict[str, Any]) -> bool:
        if not msg.get("cache", True):
            return False
        if self._model_arch.get(model, "mock") == "mock":
            return True
        inp = msg.get("inputs")
        # Only deterministic (greedy) generations are safe to serve from cache.
        return isinstance(inp, dict) and float(inp.get("temperature", 0.0)) == 0.0

    async def handle_request(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        self.stats["requests"] += 1
        rid = msg.get("request_id") or new_request_id()
        tr = self.tracer
        tr.mark(rid, "coord.recv")
        model = msg.get("model")
        inputs = msg.get("inputs")
        if not model or inputs is None:
            self.stats["errors"] += 1
            return {"error": "Missing required fields: model and inputs are required", "success": False}
        version = str(msg.get("version") or self.registry.latest_version(model) or DEFAULT_VERSION)
        if self.registry.get_model_version(model, version) is None:
            self.stats["errors"] += 1
            return {"error": f"Model '{model}' version '{version}' not registered", "success": False}
        ckey = self._cache_key(model, version, inputs) if self._cacheable(model, msg) else None
        if ckey is not None:
            hit = self.cache.get(ckey)
            if hit is not None:
                self.stats["cache_hits"] += 1
                tr.mark(rid, "coord.reply")
                return dict(hit, cached=True, request_id=rid)
        key = str(msg.get("request_key") or rid)
        shard = self.router.route_request(model, version, key)
        if shard is None:
            self.stats["errors"] += 1
            return {"error": f"no healthy shard for {model}:{version}", "success": False}
        tr.mark(rid, "coord.routed")
        vkey = f"{version}#{shard.shard_id}"
        try:
            if self.batcher.try_direct(model, vkey):
                # an idle shard: dispatch this request itself, no batch task / future in between (the lone
                # request's latency path); requests arriving meanwhile still batch behind it
                try:
                    tr.mark(rid, "coord.dispatch")
                    # one deadline over every retry (the batch path bounds its future the same way)
                    resp = await self._send(model, version, shard.shard_id, key,
                                            {"op": "infer", "model": model, "inputs": inputs, "request_id": rid},
                                            deadline=time.monotonic() + self.request_timeout_s)
                finally:
                    self.batcher.release_direct(model, vkey)
            else:
                fut = await self.batcher.add_request(model, vkey, {"inputs": inputs, "request_id": rid, "key": key})
                resp = await asyncio.wait_for(fut, self.request_timeout_s)
        except Exception as e:
            self.stats["errors"] += 1
            return {"error": str(e) or type(e).__name__, "success": False, "request_id": rid}
        tr.mark(rid, "coord.reply")
        if resp.get("success") and ckey is not None:
            self.cache.set(ckey, {k: v for k, v in resp.items() if k != "request_id"})
        if not resp.get("success"):
            self.stats["errors"] += 1
        resp.setdefault("request_id", rid)
        return resp

    async def handle_stream(self, msg: Dict[str, Any], emit) -> Dict[str, Any]:
        """Streamed request: routed like any other (hash shard → LB), bypassing the batcher and the
        response cache; the worker's token-delta frames are relayed as they arrive. A failed worker
        is retried on the next candidate only while no token has been relayed."""
        self.stats["requests"] += 1
        rid = msg.get("request_id") or new_request_id()
        model, inputs = msg.get("model"), msg.get("inputs")
        version = str(msg.get("version") or self.registry.latest_version(model) or DEFAULT_VERSION)
        if not model or self.registry.get_model_version(model, version) is None:
            self.stats["errors"] += 1
            return {"error": f"Model '{model}' version '{version}' not registered", "success": False}
        key = str(msg.get("request_key") or rid)
        shard = self.router.route_request(model, version, key)
        if shard is None:
            self.stats["errors"] += 1
            return {"error": f"no healthy shard for {model}:{version}", "success": False}
        lb = self._lb(model, version)
        wmsg = {"op": "infer", "model": model, "inputs": inputs, "request_id": rid}
        last_err = "no worker available"
        cost = request_cost(inputs)
        for i, (wid, addr) in enumerate(self._candidates(model, version, shard.shard_id, key, cost)):
            if i > self.max_retries:
                break
            relayed = False
            try:
                async with lb.track(wid, cost) as seq:
                    async for frame in self.rpc.stream(addr, dict(wmsg, lb=lb.token, lb_seq=seq),
                                                       timeout=self.request_timeout_s):
                        if isinstance(frame, dict) and frame.get("done") is False:
                            relayed = True
                            await emit(frame)
                            continue
                        self.router.mark_worker_success(wid)
                        if isinstance(frame, dict):
                            lb.observe(wid, frame.pop("engine_load", None))
                            frame.setdefault("request_id", rid)
                        return frame
            except (RPCError, OSError, asyncio.TimeoutError) as e:
                last_err = f"{wid}: {e}"
                self.router.mark_worker_failure(wid)
                if relayed:
                    break
                self.stats["retries"] += 1
        self.stats["errors"] += 1
        return {"error": last_err, "success": False, "request_id": rid, "done": True}

    # ------------------------------------------------------------ dispatch
    def _dispatch_mode(self, model: str) -> str:
        if self.dispatch_override:
            return self.dispatch_override
        return "batch" if self._model_arch.get(model, "mock") == "mock" else "stream"

    def _candidates(self, model: str, version: str, shard_id: int, key: str, cost=None):
        """Ordered worker candidates, generated lazily (the fallbacks are only computed after a failure):
        LB choice in the routed shard first, then the shard's other healthy workers, then other healthy
        shards by key affinity. ``cost``: (prompt tokens, output tokens) for the least_latency score."""
        lb = self._lb(model, version)
        seen: List[Tuple[str, str]] = []
        first = lb.pick(group=str(shard_id), cost=cost)
        if first:
            seen.append(first)
            yield first
        for w, addr in list(lb.workers.items()):
            if lb.groups.get(w) == str(shard_id) and lb.is_healthy(w) and (w, addr) not in seen:
                seen.append((w, addr))
                yield w, addr
        others = [s for s in self.router.healthy_shards(model, version) if s.shard_id != shard_id]
        others.sort(key=lambda s: -rendezvous_score(key, s.shard_id))
        for s in others:
            p = lb.pick(group=str(s.shard_id), cost=cost)
            if p and p not in seen:
                seen.append(p)
                yield p

    async def _send(self, model: str, version: str, shard_id: int, key: str, msg: Dict[str, Any],
                    deadline: Optional[float] = None) -> Dict[str, Any]:
        """Send to the routed worker, retrying on the next candidates. ``deadline`` (time.monotonic())
        bounds all attempts together: each one gets only the time that is left."""
        lb = self._lb(model, version)
        last_err = "no worker available"
        tried = 0
        if deadline is None:
            deadline = time.monotonic() + self.request_timeout_s
        cost = request_cost(msg.get("inputs")) if msg.get("op") == "infer" else None
        for wid, addr in self._candidates(model, version, shard_id, key, cost):
            if tried > self.max_retries:
                break
            left = deadline - time.monotonic()
            if left <= 0:
                last_err = f"request timed out after {self.request_timeout_s:g} s"
                break
            if tried:
                self.stats["retries"] += 1
            tried += 1
            try:
                async with lb.track(wid, cost) as seq:
                    rep = await self.rpc.call(addr, dict(msg, lb=lb.token, lb_seq=seq) if cost else msg,
                                              timeout=min(self.request_timeout_s, left))
                    if not isinstance(rep, dict):
                        raise RPCError("malformed reply")
                    lb.observe(wid, rep.pop("engine_load", None))
                    if not rep.get("success") and rep.get("retryable"):
                        raise RPCError(rep.get("error", "worker error"))
                self.router.mark_worker_success(wid)
                return rep
            except (RPCError, OSError, asyncio.TimeoutError) as e:
                last_err = f"{wid}: {e}"
                self.router.mark_worker_failure(wid)
                logger.warning("dispatch to %s failed (%s); retrying", wid, e)
        return {"error": last_err, "success": False}

    async def _batch_callback(self, model: str, vkey: str, items: List[Dict[str, Any]]) -> List[Any]:
        version, _, sid = vkey.partition("#")
        shard_id = int(sid)
        key = items[0]["key"]
        for it in items:
            self.tracer.mark(it["request_id"], "coord.dispatch")
        if self._dispatch_mode(model) == "batch":
            rep = await self._send(model, version, shard_id, key,
                                   {"op": "infer_batch", "model": model,
                                    "inputs_list": [it["inputs"] for it in items]})
            if not rep.get("success"):
                return [dict(rep) for _ in items]
            outs = rep["outputs_list"]
            return [{"model": model, "outputs": o, "worker_id": rep.get("worker_id"), "success": True}
                    for o in outs]
        deadline = time.monotonic() + self.request_timeout_s
        return [self._send(model, version, shard_id, it["key"],
                           {"op": "infer", "model": model, "inputs": it["inputs"], "request_id": it["request_id"]},
                           deadline=deadline)
                for it in items]

    # ---------------------------------------------------------------- stats
    async def get_stats(self) -> Dict[str, Any]:
        return {
            "coordinator": dict(self.stats),
            "cache": self.cache.get_stats(),
            "batcher": await self.batcher.get_stats(),
            "router": self.router.get_stats(),
            "load_balancers": {k: lb.get_all_stats() for k, lb in self.lbs.items()},
            "latency": self.tracer.summary("coord.recv", "coord.reply"),
            "workers": {w: self.router.get_worker_info(w) for w in self.router.workers},
        }

    def healthy_worker_count(self) -> int:
        return sum(1 for w in self.router.workers.values() if w.health == WorkerHealth.HEALTHY)


def build_arg_parser():
    import argparse

    p = argparse.ArgumentParser(description="Coordinator (front door)")
    p.add_argument("--listen-host", default="127.0.0.1")
    p.add_argument("--listen-port", type=int, default=9000)
    p.add_argument("--worker", action="append", default=[], help="host:port of a worker (repeatable)")
    p.add_argument("--config", default=None, help="YAML deployment config (examples/demo_config.yaml)")
    p.add_argument("--strategy", default=None,
                   choices=[s.value for s in LoadBalancerStrategy])
    p.add_argument("--max-batch-size", type=int, default=None)
    p.add_argument("--max-latency-ms", type=float, default=None)
    p.add_argument("--dispatch", default=None, choices=["batch", "stream"])
    p.add_argument("--port-file", default=None)
    p.add_argument("--procs", type=int, default=1,
                   help="coordinator processes sharing the listening port (SO_REUSEPORT); registrations are "
                        "forwarded between them")
    return p


def _configure(args) -> DeploymentConfig:
    cfg = DeploymentConfig.from_yaml(args.config) if args.config else DeploymentConfig()
    cfg.listen_host = args.listen_host or cfg.listen_host
    cfg.listen_port = args.listen_port if args.listen_port is not None else cfg.listen_port
    if args.strategy:
        cfg.strategy = args.strategy
    if args.max_batch_size:
        cfg.batch_max_size = args.max_batch_size
    if args.max_latency_ms:
        cfg.batch_max_latency_ms = args.max_latency_ms
    return cfg


def _child_main(ns: Dict[str, Any], conn) -> None:
    """One of --procs coordinator processes: serve the shared port, report the private peer address,
    learn the siblings' addresses, add the static workers, then serve until terminated."""
    import argparse

    async def run():
        setup_logging()
        args = argparse.Namespace(**ns)
        cfg = _configure(args)
        coord = Coordinator.from_config(cfg)
        coord.reuse_port = True
        coord.dispatch_override = args.dispatch
        await coord.start()
        conn.send(await coord.start_peer_server())
        loop = asyncio.get_running_loop()
        coord.peer_addrs = await loop.run_in_executor(None, conn.recv)
        addrs = list(args.worker) + [w.address for w in cfg.workers]
        await asyncio.gather(*(coord.add_static_worker(a) for a in addrs))
        conn.send("ready")
        try:
            await asyncio.Event().wait()
        finally:
            await coord.stop()

    with contextlib.suppress(KeyboardInterrupt):
        asyncio.run(run())


def run_multi(args) -> None:
    """Parent of --procs N coordinator processes on one port."""
    import multiprocessing as mp
    import signal
    import socket

    port = args.listen_port
    if not port:  # pick a free port for all of them
        s = socket.socket()
        s.bind((args.listen_host, 0))
        port = s.getsockname()[1]
        s.close()
    ns = dict(vars(args), listen_port=port)
    ctx = mp.get_context("spawn")
    pipes, procs = [], []
    for _ in range(args.procs):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_child_main, args=(ns, b), daemon=True)
        p.start()
        pipes.append(a)
        procs.append(p)
    peers = [a.recv() for a in pipes]
    for i, a in enumerate(pipes):
        a.send([x for j, x in enumerate(peers) if j != i])
    for a in pipes:
        assert a.recv() == "ready"
    if args.port_file:
        with open(args.port_file + ".tmp", "w") as f:
            f.write(str(port))
        os.replace(args.port_file + ".tmp", args.port_file)
    print(f"Coordinator x{args.procs} listening on {args.listen_host}:{port}", flush=True)

    def stop(*_):
        for p in procs:
            p.terminate()
    signal.signal(signal.SIGTERM, stop)
    try:
        for p in procs:
            p.join()
    except KeyboardInterrupt:
        stop()


async def main(argv=None) -> None:
    setup_logging()
    args = build_arg_parser().parse_args(argv)
    cfg = _configure(args)
    coord = Coordinator.from_config(cfg)
    coord.dispatch_override = args.dispatch
    port = await coord.start()
    addrs = list(args.worker) + [w.address for w in cfg.workers]
    await asyncio.gather(*(coord.add_static_worker(a) for a in addrs))
    if args.port_file:
        with open(args.port_file + ".tmp", "w") as f:
            f.write(str(port))
        os.replace(args.port_file + ".tmp", args.port_file)
    print(f"Coordinator listening on {cfg.listen_host}:{port}", flush=True)
    try:
        await asyncio.Event().wait()
    finally:
        await coord.stop()


if __name__ == "__main__":
    _args = build_arg_parser().parse_args()
    if _args.procs > 1:
        run_multi(_args)
    else:
        with contextlib.suppress(KeyboardInterrupt):
            asyncio.run(main())
