"""
Request batcher — the admission front of the serving path.

Same API as `/root/reference/src/batcher.py:37-269`: requests are buffered per
``"{model}:{version}"`` key and flushed when ``max_batch_size`` requests are
waiting or ``max_latency_ms`` has passed since the first one arrived; the
injected ``batch_callback(model, version, inputs_list)`` produces one result
per input.

On MI355X the callback is usually "submit these prompts to the worker's
continuous-batching engine" (:class:`src.engine.async_engine.AsyncLLMEngine`),
so the flush policy here only bounds *admission* latency: once admitted, a
request joins the running decode batch on the next engine iteration and
leaves it the moment it finishes. To support that, a callback may return a
list of awaitables; each request's future is then resolved as soon as *its*
awaitable completes (streaming completion), instead of waiting for the whole
batch.

Defects fixed: the callback never runs while the lock is
held (the reference's timer path did, `batcher.py:155-166`, so a re-entrant
``add_request`` deadlocked); a size-triggered flush does not make the caller
wait for the model (`batcher.py:146-147`); ``get_stats`` has no duplicate key.
Optional ``coalesce``/``split`` hooks implement "coalesce compatible inputs
into one payload and decompress outputs" (`README.md:80`).
"""

from __future__ import annotations

import asyncio
import contextlib
import inspect
import logging
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Awaitable, Callable, Dict, List, Optional

logger = logging.getLogger(__name__)

BatchCallback = Callable[[str, str, List[Any]], Awaitable[List[Any]]]


@dataclass
class BatchedRequest:
    request_id: str
    model_name: str
    version: str
    inputs: Any
    created_at: float
    future: asyncio.Future = field(default=None)  # type: ignore[assignment]


@dataclass
class Batch:
    model_name: str
    version: str
    requests: List[BatchedRequest]
    created_at: float
    max_batch_size: int
    max_latency: float
    last_arrival: float = 0.0   # time.monotonic() of the latest request (idle-gap flush)


class Batcher:
    def __init__(
        self,
        max_batch_size: int = 32,
        max_latency_ms: float = 100.0,
        batch_callback: Optional[BatchCallback] = None,
        coalesce: Optional[Callable[[List[Any]], Any]] = None,
        split: Optional[Callable[[Any, int], List[Any]]] = None,
        max_inflight_batches: Optional[int] = None,
        eager_when_idle: bool = False,
        idle_flush_ms: Optional[float] = None,
    ):
        if max_batch_size < 1:
            raise ValueError("max_batch_size must be at least 1")
        if max_latency_ms <= 0:
            raise ValueError("max_latency_ms must be greater than 0")
        self.max_batch_size = max_batch_size
        self.max_latency = max_latency_ms / 1000.0
        # idle_flush_ms: a partial batch is also flushed once no request has arrived for this long
        # (max_latency stays the bound). Closed-loop clients that are all waiting on this batch send nothing
        # until it returns: without it, every such batch (e.g. 16 clients per coordinator process under
        # SO_REUSEPORT, batch size 32) waited the full max_latency.
        self.idle_flush = (idle_flush_ms / 1000.0) if idle_flush_ms else None
        self.batch_callback = batch_callback
        self.coalesce = coalesce
        self.split = split
        self._batches: Dict[str, Batch] = {}
        self._flush_tasks: Dict[str, asyncio.Task] = {}
        self._inflight: set = set()
        self._sem = asyncio.Semaphore(max_inflight_batches) if max_inflight_batches else None
        # eager_when_idle: a request for a key with nothing in flight is dispatched at once
        # (no max_latency wait when the backend is idle); later arrivals batch up behind it.
        self.eager_when_idle = eager_when_idle
        self._inflight_by_key: Dict[str, int] = {}
        self._running = False
        self._lock = asyncio.Lock()
        self.total_batches = 0
        self.total_requests = 0
        self.total_batched_requests = 0
        self.total_errors = 0
        self._wait_time_total = 0.0

    # -------------------------------------------------------------- lifecycle
    async def start(self) -> None:
        if self._running:
            logger.warning("Batcher is already running")
            return
        self._running = True

    async def stop(self) -> None:
        """Stop accepting requests, flush what is pending and wait for every
        in-flight batch (reference `batcher.py:70-100` drains too)."""
        if not self._running:
            return
        self._running = False
        async with self._lock:
            timers = list(self._flush_tasks.values())
            pending = [(k, b, list(b.requests)) for k, b in self._batches.items() if b.requests]
            self._flush_tasks.clear()
            self._batches.clear()
        for t in timers:
            if not t.done():
                t.cancel()
                with contextlib.suppress(asyncio.CancelledError):
                    await t
        for key, batch, reqs in pending:
            await self._process_batch(key, batch, reqs)
        if self._inflight:
            await asyncio.gather(*list(self._inflight), return_exceptions=True)

    @property
    def running(self) -> bool:
        return self._running

    # -------------------------------------------------------------- admission
    async def add_request(
        self,
        model_name: str,
        version: str,
        inputs: Any,
        request_id: Optional[str] = None,
    ) -> asyncio.Future:
        if not self._running:
            raise RuntimeError("Batcher is not running")
        loop = asyncio.get_running_loop()
        req = BatchedRequest(
            request_id=request_id or str(uuid.uuid4()),
            model_name=model_name,
            version=version,
            inputs=inputs,
            created_at=time.time(),
            future=loop.create_future(),
        )
        key = f"{model_name}:{version}"
        to_flush: Optional[List[BatchedRequest]] = None
        async with self._lock:
            batch = self._batches.get(key)
            if batch is None and self.eager_when_idle and not self._inflight_by_key.get(key):
                self.total_requests += 1
                eager = Batch(model_name, version, [req], time.time(), self.max_batch_size, self.max_latency)
                self._spawn(key, eager, [req])
                return req.future
            if batch is None:
                batch = Batch(model_name, version, [], time.time(), self.max_batch_size, self.max_latency)
                self._batches[key] = batch
                self._flush_tasks[key] = asyncio.create_task(self._timer(key, batch))
            batch.requests.append(req)
            batch.last_arrival = time.monotonic()
            self.total_requests += 1
            if len(batch.requests) >= self.max_batch_size:
                to_flush = self._detach(key, batch)
        if to_flush:
            self._spawn(key, batch, to_flush)
        return req.future

    def try_direct(self, model_name: str, version: str) -> bool:
        """Claim an idle key (nothing queued, nothing in flight) for ONE request dispatched by the caller
        itself, without a batch task or future: the latency path of a lone request. While it is in
        flight the key counts as busy, so concurrent requests still form batches behind it.
        Pair with :meth:`release_direct`. No await inside: atomic on the event loop."""
        key = f"{model_name}:{version}"
        if not (self._running and self.eager_when_idle) or key in self._batches or self._inflight_by_key.get(key):
            return False
        # the direct request counts against max_inflight_batches like a batch does: refuse when every
        # slot is taken (the caller then queues normally), else take one without suspending
        if self._sem is not None and not self._try_acquire_slot():
            return False
        self._inflight_by_key[key] = 1
        self.total_requests += 1
        self.total_batches += 1
        return True

    def release_direct(self, model_name: str, version: str) -> None:
        key = f"{model_name}:{version}"
        self._inflight_by_key[key] = self._inflight_by_key.get(key, 1) - 1
        if self._sem is not None:
            self._sem.release()

    def _try_acquire_slot(self) -> bool:
        """Non-blocking acquire of the in-flight semaphore (asyncio.Semaphore has none): when it is not
        locked, acquire() completes without suspending, so drive that coroutine to its end here."""
        if self._sem.locked():
            return False
        coro = self._sem.acquire()
        try:
            coro.send(None)
        except StopIteration:
            return True
        coro.close()  # it suspended (cannot happen while unlocked): leave the semaphore as it was
        return False

    def _detach(self, key: str, batch: Batch) -> List[BatchedRequest]:
        """Take the batch's requests and forget the batch. Caller holds the lock."""
        reqs = list(batch.requests)
        batch.requests.clear()
        if self._batches.get(key) is batch:
            del self._batches[key]
        t = self._flush_tasks.pop(key, None)
        if t is not None and t is not asyncio.current_task() and not t.done():
            t.cancel()
        return reqs

    def _spawn(self, key: str, batch: Batch, reqs: List[BatchedRequest]) -> None:
        task = asyncio.create_task(self._process_batch(key, batch, reqs))
        self._inflight.add(task)
        self._inflight_by_key[key] = self._inflight_by_key.get(key, 0) + 1

        def done(t, key=key):
            self._inflight.discard(t)
            self._inflight_by_key[key] -= 1

        task.add_done_callback(done)

    async def _timer(self, key: str, batch: Batch) -> None:
        try:
            if self.idle_flush is None:
                await asyncio.sleep(batch.max_latency)
            else:  # flush at max_latency, or earlier once arrivals have paused for idle_flush
                t_end = time.monotonic() + batch.max_latency
                while True:
                    now = time.monotonic()
                    wake = min(t_end, (batch.last_arrival or now) + self.idle_flush)
                    if wake <= now:
                        break
                    await asyncio.sleep(wake - now)
        except asyncio.CancelledError:
            return
        async with self._lock:
            if self._batches.get(key) is not batch or not batch.requests:
                return
            reqs = self._detach(key, batch)
        # Outside the lock: the callback may call add_request again.
        self._spawn(key, batch, reqs)

    async def flush(self) -> None:
        """Flush every pending batch now (does not wait for the results)."""
        async with self._lock:
            work = [(k, b, self._detach(k, b)) for k, b in list(self._batches.items()) if b.requests]
        for k, b, reqs in work:
            self._spawn(k, b, reqs)

    # ------------------------------------------------------------- execution
    async def _process_batch(self, key: str, batch: Batch, reqs: List[BatchedRequest]) -> None:
        if not reqs:
            return
        self.total_batches += 1
        self.total_batched_requests += len(reqs)
        now = time.time()
        self._wait_time_total += sum(now - r.created_at for r in reqs)
        if self.batch_callback is None:
            err = RuntimeError("No batch callback configured")
            for r in reqs:
                if not r.future.done():
                    r.future.set_exception(err)
            return
        sem = self._sem or contextlib.nullcontext()
        try:
            async with sem:  # type: ignore[attr-defined]
                inputs = [r.inputs for r in reqs]
                if self.coalesce is not None:
                    payload = self.coalesce(inputs)
                    out = await self.batch_callback(batch.model_name, batch.version, payload)
                    results = self.split(out, len(reqs)) if self.split else out
                else:
                    results = await self.batch_callback(batch.model_name, batch.version, inputs)
                if len(results) != len(reqs):
                    raise ValueError(f"Batch callback returned {len(results)} results but expected {len(reqs)}")
                waits = []
                for r, res in zip(reqs, results):
                    if inspect.isawaitable(res):
                        waits.append(self._chain(r, res))
                    elif not r.future.done():
                        r.future.set_result(res)
                if waits:
                    await asyncio.gather(*waits)
        except Exception as e:  # every request of the batch sees the failure
            self.total_errors += 1
            logger.exception("Error processing batch %s", key)
            for r in reqs:
                if not r.future.done():
                    r.future.set_exception(e)

    @staticmethod
    async def _chain(req: BatchedRequest, aw: Awaitable) -> None:
        try:
            res = await aw
        except Exception as e:
            if not req.future.done():
                req.future.set_exception(e)
            return
        if not req.future.done():
            req.future.set_result(res)

    # ----------------------------------------------------------------- stats
    async def get_stats(self) -> Dict[str, Any]:
        async with self._lock:
            nonempty = [b for b in self._batches.values() if b.requests]
            pending_requests = sum(len(b.requests) for b in nonempty)
        return {
            "total_batches": self.total_batches,
            "total_requests": self.total_requests,
            "total_batched_requests": self.total_batched_requests,
            "total_errors": self.total_errors,
            "pending_batches": len(nonempty),
            "pending_batches_count": len(nonempty),
            "pending_requests": pending_requests,
            "inflight_batches": len(self._inflight),
            "avg_batch_size": (self.total_batched_requests / self.total_batches) if self.total_batches else 0.0,
            "avg_admission_wait_ms": (1e3 * self._wait_time_total / self.total_batched_requests)
            if self.total_batched_requests else 0.0,
            "max_batch_size": self.max_batch_size,
            "max_latency_ms": self.max_latency * 1000.0,
        }
