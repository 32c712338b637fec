"""
Worker: one serving process, owning one GPU (or one TP rank group entry) and
the model sessions on it.

Public API kept from `/root/reference/src/worker.py:26-209`: ``Worker(worker_id,
host, port)``, ``await start() -> port``, ``await shutdown()``,
``load_model(ModelConfig)``, ``unload_model(name)``, ``get_metrics()`` and the
in-process ``await _process_request(dict)`` the reference demos call. The wire
request is still ``{"model", "inputs", ...}`` and the reply
``{"model","outputs","worker_id","success"}`` / ``{"error","success":false}``
(`worker.py:135-162`).

What is new:

* the model behind ``predict`` is either the reference's mock
  (:class:`FakeModel`, ``arch="mock"``) or a real MI355X session
  (:class:`src.engine.backend.LLMBackend`: Llama-3 / Mixtral on PyTorch-ROCm
  with hand-written HIP kernels, paged KV in HBM, continuous batching);
* framed messages on persistent connections (legacy unframed JSON still served);
* an ``op`` verb: ``infer`` (default), ``infer_batch``, ``health``, ``metrics``,
  ``load_model``, ``unload_model``, ``kv_export``/``kv_import`` (disaggregated
  prefill → decode), ``stats``; a health probe is answered cheaply and not
  counted as a request (the reference counted probes, `worker.py:87`);
* a registration handshake with the coordinator (`README.md:85`);
* ``python src/worker.py`` works as well as ``python -m src.worker``, and
  ``--model`` / ``--arch`` / ``--preset`` select what to serve (`README.md:108`).
"""

from __future__ import annotations

import asyncio
import contextlib
import logging
import os
import signal
import sys
import time
from typing import Any, Dict, List, Optional

if __package__ in (None, ""):  # `python src/worker.py`
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import psutil  # noqa: E402

from src.config import ModelConfig  # noqa: E402
from src.mock_models import FakeModel  # noqa: E402
from src.rpc import RPCClient  # noqa: E402
from src.utils import GLOBAL_TRACER, setup_logging  # noqa: E402
from src.utils.frameserver import start_frame_server  # noqa: E402

logger = logging.getLogger(__name__)


def make_backend(config: ModelConfig):
    """Instantiate the backend for ``config.arch``."""
    if config.arch in ("mock", "fake", "echo"):
        return FakeModel(config)
    if config.arch in ("llama", "mixtral"):
        from src.engine.backend import LLMBackend

        return LLMBackend(config)
    raise ValueError(f"unknown model arch {config.arch!r}")


class Worker:
    def __init__(self, worker_id: str, host: str = "0.0.0.0", port: int = 0,
                 coordinator: Optional[str] = None, metadata: Optional[Dict[str, Any]] = None,
                 install_signal_handlers: bool = True):
        self.worker_id = worker_id
        self.host = host
        self.port = port
        self.coordinator = coordinator
        self.metadata = metadata or {}
        self.install_signal_handlers = install_signal_handlers
        self.models: Dict[str, Any] = {}
        self._lb_seen: Dict[str, int] = {}  # balancer token -> highest dispatch sequence number received
        self.server: Optional[asyncio.AbstractServer] = None
        self._stop_event = asyncio.Event()
        self._start_time = time.time()
        self._request_count = 0
        self._error_count = 0
        self._probe_count = 0
        self._active = 0
        self._conns: set = set()
        self._bg: set = set()      # background tasks (signal shutdown): held so they are not collected
        self._waiters = 0
        self._tracer = GLOBAL_TRACER
        self._process = psutil.Process()

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> int:
        loop = asyncio.get_running_loop()
        if self.install_signal_handlers:
            for sig in (signal.SIGTERM, signal.SIGINT):
                with contextlib.suppress(NotImplementedError, RuntimeError, ValueError):
                    loop.add_signal_handler(sig, self._on_signal, sig)
        for m in self.models.values():
            if hasattr(m, "start"):
                await m.start()
        # protocol-level framing (src/utils/frameserver.py); an idle connection is dropped after IDLE_TIMEOUT_S
        # (the timer stops while a request is being served: a long streamed generation is not idle)
        self.server = await start_frame_server(self.handle_message, self.host, self.port, backlog=4096,
                                               idle_timeout=self.IDLE_TIMEOUT_S, conns=self._conns,
                                               on_error=self._on_protocol_error)
        self.port = self.server.sockets[0].getsockname()[1]
        logger.info("Worker %s listening on %s:%d", self.worker_id, self.host, self.port)
        if self.coordinator:
            asyncio.create_task(self._register_with_coordinator())
        return self.port

    def _on_protocol_error(self, exc: BaseException) -> None:
        """A request the framing layer rejected (bad frame, malformed JSON): counted as a request and an error,
        as the reference's handler counted a failed json.loads (`/root/reference/src/worker.py:87,99-101`)."""
        self._request_count += 1
        self._error_count += 1

    @property
    def address(self) -> str:
        host = "127.0.0.1" if self.host in ("0.0.0.0", "") else self.host
        return f"{host}:{self.port}"

    async def _register_with_coordinator(self, attempts: int = 60) -> bool:
        client = RPCClient(max_idle_per_host=1)
        msg = {
            "op": "register",
            "worker_id": self.worker_id,
            "address": self.address,
            "models": {name: getattr(m, "config", ModelConfig(name, "")).to_dict()
                       for name, m in self.models.items()},
            "metadata": self.metadata,
        }
        try:
            for i in range(attempts):
                try:
                    rep = await client.call(self.coordinator, msg, timeout=5.0)
                    if isinstance(rep, dict) and rep.get("success"):
                        logger.info("Registered with coordinator %s", self.coordinator)
                        return True
                except Exception as e:  # coordinator not up yet
                    logger.debug("registration attempt %d failed: %s", i, e)
                await asyncio.sleep(min(0.25 * (i + 1), 2.0))
            return False
        finally:
            client.close()

    def _on_signal(self, sig) -> None:
        t = asyncio.get_running_loop().create_task(self.shutdown(sig))
        self._bg.add(t)
        # a SystemExit raised by shutdown() leaves the loop anyway: retrieve it on the task too, so asyncio
        # does not log "Task exception was never retrieved" at exit (round 3's SIGTERM noise)
        t.add_done_callback(lambda t: (self._bg.discard(t), t.cancelled() or t.exception()))

    async def shutdown(self, sig=None) -> None:
        if sig:
            logger.info("Received signal %s, shutting down", getattr(sig, "name", sig))
        if self.server:
            self.server.close()
            for w in list(self._conns):
                with contextlib.suppress(Exception):
                    w.close()
            with contextlib.suppress(Exception):
                await asyncio.wait_for(self.server.wait_closed(), 2.0)
            self.server = None
        for name in list(self.models):
            m = self.models[name]
            if hasattr(m, "stop"):
                with contextlib.suppress(Exception):
                    await m.stop()
            self.unload_model(name)
        self._stop_event.set()
        if sig and not self._waiters:
            # the reference exits the process on a signal (`/root/reference/src/worker.py:80-82`); a caller
            # that awaits wait_closed() (our main) returns normally instead
            sys.exit(0)

    async def wait_closed(self) -> None:
        self._waiters += 1
        try:
            await self._stop_event.wait()
        finally:
            self._waiters -= 1

    IDLE_TIMEOUT_S = 3600.0

    async def handle_message(self, msg: Any, emit=None) -> Dict[str, Any]:
        """One RPC. ``emit``: writes an intermediate frame on the caller's connection — streamed
        generations (``inputs["stream"]``) send token deltas through it before the final reply."""
        if not isinstance(msg, dict):
            self._request_count += 1
            self._error_count += 1
            return {"error": "Request must be a JSON object", "success": False}
        op = msg.get("op", "infer")
        if op == "health":
            self._probe_count += 1
            failed = self.failed_models()
            lb = msg.get("lb")
            return {"success": not failed, "worker_id": self.worker_id, "load": self.load(), "failed_models": failed,
                    "engine_load": self.engine_load(msg.get("model"), lb),
                    # one report per model: a per-model balancer scores this worker by its own model's engine
                    "engine_loads": {n: self.engine_load(n, lb) for n in self.models
                                     if hasattr(self.models[n], "load_report")},
                    "models": list(self.models),
                    "archs": {n: getattr(getattr(m, "config", None), "arch", "mock") for n, m in self.models.items()}}
        if op == "metrics":
            return {"success": True, "metrics": self.get_metrics()}
        if op == "load_model":
            try:
                ok = await asyncio.get_running_loop().run_in_executor(
                    None, self.load_model, ModelConfig.from_dict(msg["config"]))
                m = self.models.get(msg["config"]["model_name"])
                if ok and m is not None and hasattr(m, "start"):
                    await m.start()
                return {"success": ok}
            except Exception as e:
                return {"error": str(e), "success": False}
        if op == "unload_model":
            name = msg.get("model")
            m = self.models.get(name)
            if m is not None and hasattr(m, "stop"):
                await m.stop()
            return {"success": self.unload_model(name)}
        if op == "abort":
            m = self.models.get(msg.get("model"))
            ok = m is not None and hasattr(m, "abort_request") and m.abort_request(str(msg.get("request_id")))
            return {"success": bool(ok), "request_id": msg.get("request_id")}
        if op in ("infer", "infer_batch"):
            self._request_count += 1
            self._active += 1
            lb, lb_seq = msg.get("lb"), msg.get("lb_seq")
            if isinstance(lb, str) and isinstance(lb_seq, int):  # which of a balancer's dispatches have arrived
                if lb_seq > self._lb_seen.get(lb, 0):
                    if len(self._lb_seen) > 256 and lb not in self._lb_seen:
                        self._lb_seen.clear()
                    self._lb_seen[lb] = lb_seq
            try:
                resp = await (self._process_batch(msg) if op == "infer_batch" else self._process_request(msg, emit))
            finally:
                self._active -= 1
            if not resp.get("success"):
                self._error_count += 1
            el = self.engine_load(msg.get("model"), lb)
            if el is not None:  # piggybacked for the coordinator's load balancer (least_latency)
                resp["engine_load"] = el
            return resp
        if op in ("kv_export", "kv_import", "kv_channel", "kv_reserve", "kv_release", "engine_stats"):
            m = self.models.get(msg.get("model"))
            if m is None or not hasattr(m, "handle_op"):
                return {"error": f"op {op} unsupported for model {msg.get('model')!r}", "success": False}
            try:
                return await m.handle_op(op, msg)
            except Exception as e:
                return {"error": str(e), "success": False}
        return {"error": f"unknown op {op!r}", "success": False}

    # ------------------------------------------------------------ inference
    async def _process_request(self, request: Dict[str, Any], emit=None) -> Dict[str, Any]:
        if not isinstance(request, dict):
            return {"error": "Request must be a JSON object", "success": False}
        model_name = request.get("model")
        inputs = request.get("inputs")
        if not model_name or inputs is None:
            return {"error": "Missing required fields: model and inputs are required", "success": False}
        model = self.models.get(model_name)
        if model is None:
            return {"error": f"Model '{model_name}' not found", "success": False}
        if model_name in self.failed_models():
            return {"error": f"model '{model_name}' engine failed on {self.worker_id}", "success": False,
                    "retryable": True}
        rid = request.get("request_id")
        try:
            if rid:
                self._tracer.mark(rid, "worker.recv")
            stream = emit is not None and isinstance(inputs, dict) and inputs.get("stream") and \
                hasattr(model, "predict_stream")
            if stream:
                async def emit_rid(frame):
                    await emit(dict(frame, request_id=rid) if rid else frame)

                outputs = await model.predict_stream(inputs, emit_rid, request_id=rid)
            elif hasattr(model, "abort_request"):
                outputs = await model.predict(inputs, request_id=rid)
            else:
                outputs = await model.predict(inputs)
            if rid:
                self._tracer.mark(rid, "worker.done")
            resp = {"model": model_name, "outputs": outputs, "worker_id": self.worker_id, "success": True}
            if stream:
                resp["done"] = True
            if rid:
                resp["request_id"] = rid
            return resp
        except Exception as e:
            logger.error("Error processing request: %s", e)
            # an engine failure (not a bad input) may succeed on another replica
            return {"error": str(e), "success": False, "retryable": model_name in self.failed_models()}

    async def _process_batch(self, request: Dict[str, Any]) -> Dict[str, Any]:
        model_name = request.get("model")
        inputs_list = request.get("inputs_list")
        if not model_name or not isinstance(inputs_list, list):
            return {"error": "infer_batch needs model and inputs_list", "success": False}
        model = self.models.get(model_name)
        if model is None:
            return {"error": f"Model '{model_name}' not found", "success": False}
        try:
            if hasattr(model, "predict_batch"):
                outs = await model.predict_batch(inputs_list)
            else:
                outs = await asyncio.gather(*(model.predict(x) for x in inputs_list))
            return {"model": model_name, "outputs_list": outs, "worker_id": self.worker_id, "success": True}
        except Exception as e:
            logger.error("Error processing batch: %s", e)
            return {"error": str(e), "success": False, "retryable": model_name in self.failed_models()}

    # --------------------------------------------------------------- models
    def failed_models(self) -> List[str]:
        """Loaded models whose engine has died (GPU fault surfaced by the engine loop)."""
        return [n for n, m in self.models.items() if hasattr(m, "healthy") and not m.healthy()]

    def load_model(self, config: ModelConfig) -> bool:
        if config.model_name in self.models:
            logger.warning("Model '%s' is already loaded", config.model_name)
            return True
        try:
            self.models[config.model_name] = make_backend(config)
            logger.info("Loaded model '%s' (%s) on worker %s", config.model_name, config.arch, self.worker_id)
            return True
        except Exception:
            logger.exception("Error loading model '%s'", config.model_name)
            return False

    def unload_model(self, model_name: str) -> bool:
        m = self.models.pop(model_name, None)
        if m is None:
            return False
        with contextlib.suppress(Exception):
            m.close()
        return True

    # -------------------------------------------------------------- metrics
    def load(self) -> float:
        loads = [m.load() for m in self.models.values() if hasattr(m, "load")]
        return max(loads) if loads else float(self._active)

    def engine_load(self, model: Optional[str] = None, lb: Optional[str] = None) -> Optional[Dict[str, Any]]:
        """The engine-state report of ``model`` (default: the first model that has one), or None. ``lb``: the asking
        balancer's token — the report then says up to which of its dispatch sequence numbers it covers
        (``lb_seen``, see LoadBalancer.observe)."""
        ms = [self.models[model]] if model in self.models else list(self.models.values())
        for m in ms:
            if hasattr(m, "load_report"):
                try:
                    r = m.load_report()
                except Exception:  # noqa: BLE001 - a report must never fail a request
                    return None
                if lb is not None and lb in self._lb_seen:
                    r = dict(r, lb=lb, lb_seen=self._lb_seen[lb])
                return r
        return None

    def get_metrics(self) -> Dict[str, Any]:
        mem = self._process.memory_info()
        try:
            conns = len(self._process.net_connections())
        except Exception:
            conns = -1
        out = {
            "worker_id": self.worker_id,
            "start_time": self._start_time,
            "uptime": time.time() - self._start_time,
            "request_count": self._request_count,
            "error_count": self._error_count,
            "probe_count": self._probe_count,
            "active_requests": self._active,
            "loaded_models": list(self.models.keys()),
            "model_metrics": {n: m.get_metrics() for n, m in self.models.items()},
            "memory_usage_mb": mem.rss / (1024 * 1024),
            "cpu_percent": self._process.cpu_percent(),
            "thread_count": self._process.num_threads(),
            "connections": conns,
        }
        out.update(self.metadata)
        return out


def build_arg_parser():
    import argparse

    p = argparse.ArgumentParser(description="MI355X inference worker")
    p.add_argument("--worker-id", default=None, help="Unique worker ID (default: worker-<port>)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=0, help="0 = OS-assigned")
    p.add_argument("--model", default="test-model", help="name to serve the model under")
    p.add_argument("--arch", default="mock", choices=["mock", "llama", "mixtral"])
    p.add_argument("--preset", default=None, help="architecture preset, e.g. llama3-8b")
    p.add_argument("--model-path", default="")
    p.add_argument("--max-batch-size", type=int, default=32)
    p.add_argument("--max-latency-ms", type=float, default=10.0)
    p.add_argument("--max-model-len", type=int, default=4096)
    p.add_argument("--tp-size", type=int, default=1)
    p.add_argument("--moe-parallel", choices=["tp", "ep"], default="tp",
                   help="MoE under TP: split each expert (tp) or give ranks whole experts (ep)")
    p.add_argument("--sequence-parallel", action="store_true",
                   help="TP prefill: token-sharded norms, reduce-scatter/all-gather instead of all-reduce")
    p.add_argument("--role", default="both", choices=["both", "prefill", "decode"])
    p.add_argument("--mock-latency-ms", type=float, default=None,
                   help="FakeModel latency; default = reference 50-150 ms")
    p.add_argument("--no-graph", action="store_true", help="disable hipGraph decode capture")
    p.add_argument("--decode-worker", default=None,
                   help="(role=prefill) host:port of the decode worker that receives the prompt KV")
    p.add_argument("--device", default=None, help="torch device for LLM backends (default cuda:0 / cpu)")
    p.add_argument("--num-kv-blocks", type=int, default=None)
    p.add_argument("--kv-block-ttl-s", type=float, default=None, help="TTL of cached (released) KV blocks")
    p.add_argument("--kv-capacity-priority", action="store_true",
                   help="the KV pool is the constraint: decode weights in one layout (EngineConfig)")
    p.add_argument("--preproc-processes", type=int, default=0,
                   help="tokenise / detokenise text in this many separate processes (0: inline)")
    p.add_argument("--coordinator", default=None, help="host:port to register with")
    p.add_argument("--port-file", default=None, help="write the bound port here once listening")
    return p


async def main(argv=None) -> None:
    setup_logging()
    args = build_arg_parser().parse_args(argv)
    overrides: Dict[str, Any] = {}
    if args.mock_latency_ms is not None:
        overrides["latency_s"] = args.mock_latency_ms / 1000.0
    if args.decode_worker:
        overrides["decode_worker"] = args.decode_worker
    if args.device:
        overrides["device"] = args.device
    if args.kv_block_ttl_s:
        overrides["kv_block_ttl_s"] = args.kv_block_ttl_s
    if args.kv_capacity_priority:
        overrides["kv_capacity_priority"] = True
    cfg = ModelConfig(
        model_name=args.model, model_path=args.model_path, batch_size=min(8, args.max_batch_size),
        max_batch_size=args.max_batch_size, arch=args.arch, preset=args.preset, tp_size=args.tp_size,
        role=args.role, max_model_len=args.max_model_len, max_latency_ms=args.max_latency_ms,
        use_cuda_graph=not args.no_graph, num_kv_blocks=args.num_kv_blocks, overrides=overrides,
        preproc_processes=args.preproc_processes,
    )
    worker = Worker(worker_id=args.worker_id or f"worker-{os.getpid()}", host=args.host, port=args.port,
                    coordinator=args.coordinator,
                    metadata={"role": args.role, "gpu": os.environ.get("HIP_VISIBLE_DEVICES")})
    if not worker.load_model(cfg):
        raise SystemExit(f"failed to load model {cfg.model_name}")
    port = await worker.start()
    if args.port_file:
        with open(args.port_file + ".tmp", "w") as f:
            f.write(str(port))
        os.replace(args.port_file + ".tmp", args.port_file)
    print(f"Worker {worker.worker_id} started on port {port}", flush=True)
    try:
        await worker.wait_closed()
    except asyncio.CancelledError:
        pass
    finally:
        if worker.server is not None:
            await worker.shutdown()


if __name__ == "__main__":
    asyncio.run(main())
