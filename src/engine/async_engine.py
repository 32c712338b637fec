"""
AsyncLLMEngine: runs the LLMEngine step loop on a dedicated thread and hands
results back to asyncio.

The reference runs "inference" on the event loop itself (an ``asyncio.sleep``
inside the RPC handler, `/root/reference/src/worker.py:152`). A real GPU step
loop must never share the event-loop thread: here the RPC side calls
:meth:`submit` (thread-safe, returns an ``asyncio.Future``), the engine thread
drains the submission queue between steps, and each finished sequence resolves
its future via ``loop.call_soon_threadsafe``. No lock is held across an await
or across a GPU step.
"""

from __future__ import annotations

import asyncio
import logging
import queue
import threading
import time
from typing import Any, Callable, Dict, List, Optional

from src.engine.llm_engine import LLMEngine
from src.engine.sequence import Sequence
from src.preproc import SamplingParams

logger = logging.getLogger(__name__)


class AsyncLLMEngine:
    def __init__(self, engine: LLMEngine, name: str = "engine"):
        self.engine = engine
        self.name = name
        self._q: "queue.Queue" = queue.Queue()
        self._aborts: "queue.Queue" = queue.Queue()
        self._wake = threading.Event()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.error: Optional[BaseException] = None

    def start(self) -> None:
        if self._thread is not None:
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, name=f"{self.name}-loop", daemon=True)
        self._thread.start()

    def stop(self, timeout: float = 30.0) -> None:
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout)
            self._thread = None

    @property
    def running(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    def submit(self, request_id: str, prompt_ids: List[int], sampling: SamplingParams,
               loop: Optional[asyncio.AbstractEventLoop] = None, user_data: Any = None,
               on_token: Optional[Callable[[int], None]] = None) -> asyncio.Future:
        """Thread-safe; call from the event loop. The future resolves to the
        finished :class:`Sequence` (or raises if the engine failed). ``on_token(tok)`` (streaming)
        runs on the event loop for every generated token, in order, before the future resolves."""
        loop = loop or asyncio.get_running_loop()
        fut = loop.create_future()
        if self.error is not None:
            fut.set_exception(RuntimeError(f"engine failed: {self.error!r}"))
            return fut
        if on_token is not None:
            user_data = dict(user_data or {}, on_token=on_token)
        self._q.put((request_id, prompt_ids, sampling, fut, loop, user_data))
        self._wake.set()
        if self.error is not None:  # the loop died between the check above and the put
            self._fail_pending()
        return fut

    def submit_sync(self, request_id: str, prompt_ids: List[int], sampling: SamplingParams,
                    callback) -> None:
        """Non-asyncio submission: ``callback(seq_or_exception)`` runs on the engine thread."""
        self._q.put((request_id, prompt_ids, sampling, callback, None, None))
        self._wake.set()
        if self.error is not None:
            self._fail_pending()

    def abort(self, request_id: str) -> None:
        """Thread-safe: drop a queued or running request (its KV blocks are freed between steps and its
        future resolves with ``finish_reason == "abort"`` and the tokens generated so far)."""
        self._aborts.put(request_id)
        self._wake.set()

    def call(self, fn, loop: Optional[asyncio.AbstractEventLoop] = None) -> asyncio.Future:
        """Run ``fn(engine)`` on the engine thread between steps; the future
        gets its return value (used for KV import/export and stats)."""
        loop = loop or asyncio.get_running_loop()
        fut = loop.create_future()
        self._q.put(("__call__", fn, None, fut, loop, None))
        self._wake.set()
        if self.error is not None:
            self._fail_pending()
        return fut

    def _fail_pending(self) -> None:
        """After the loop died: fail every queued submission (thread-safe, idempotent)."""
        err = RuntimeError(f"engine failed: {self.error!r}")
        while True:
            try:
                rid, _, _, fut, loop, _ = self._q.get_nowait()
            except queue.Empty:
                return
            if loop is None:
                fut(err)
            else:
                loop.call_soon_threadsafe(_fail, fut, err)

    def _drain(self) -> None:
        self._drain_submissions()
        while True:  # aborts after submissions: an abort may follow its own submit in the same drain
            try:
                rid = self._aborts.get_nowait()
            except queue.Empty:
                return
            self.engine.abort(rid)

    def _drain_submissions(self) -> None:
        while True:
            try:
                rid, ids, sp, fut, loop, ud = self._q.get_nowait()
            except queue.Empty:
                return
            if rid == "__call__":
                try:
                    res = ids(self.engine)
                    loop.call_soon_threadsafe(_set, fut, res)
                except Exception as e:
                    loop.call_soon_threadsafe(_fail, fut, e)
                continue

            def done(seq: Sequence, fut=fut, loop=loop):
                if loop is None:
                    fut(seq)
                else:
                    loop.call_soon_threadsafe(_resolve, fut, seq)

            on_tok = None
            if isinstance(ud, dict) and ud.get("on_token") is not None and loop is not None:
                def on_tok(seq: Sequence, tok: int, cb=ud["on_token"], loop=loop):
                    loop.call_soon_threadsafe(cb, tok)
            try:
                if isinstance(ud, dict) and ud.get("import_packet") is not None:
                    self.engine.add_imported(ud["import_packet"], sp, on_finish=done)
                else:
                    self.engine.add_request(rid, ids, sp, on_finish=done, user_data=ud,
                                            export_kv=isinstance(ud, dict) and bool(ud.get("export_kv")),
                                            on_token=on_tok)
            except Exception as e:
                if loop is None:
                    fut(e)
                else:
                    loop.call_soon_threadsafe(_fail, fut, e)

    def _loop(self) -> None:
        eng = self.engine
        try:
            if eng.device.type == "cuda":
                # the current device is per thread: the kernels' bindings launch on the current device's
                # current stream, so a worker serving cuda:N (run.sh DISAGG exposes every GPU to every
                # worker) must select it on this thread too
                import torch

                if eng.device.index is not None:
                    torch.cuda.set_device(eng.device)
            while not self._stop.is_set():
                self._drain()
                if not eng.has_work():
                    eng.runner.idle_tick()
                    self._wake.wait(0.05)
                    self._wake.clear()
                    continue
                finished = eng.step()
                if not finished and not eng.scheduler.running:
                    # admission is being held for batching (max_latency): sleep until due
                    w = eng.scheduler.next_wakeup()
                    if w:
                        self._wake.wait(min(w, 0.01))
                        self._wake.clear()
        except BaseException as e:  # surface GPU/HIP faults to every waiter
            logger.exception("engine loop crashed")
            self.error = e
            for seq in list(eng.seqs.values()):
                if seq.on_finish is not None:
                    seq.finish_reason = "error"
                    try:
                        seq.on_finish(seq)
                    except Exception:
                        pass
            self._fail_pending()

    def stats(self) -> Dict[str, Any]:
        s = self.engine.get_stats()
        s["queue"] = self._q.qsize()
        s["alive"] = self.running
        s["error"] = repr(self.error) if self.error else None
        return s


def _resolve(fut: asyncio.Future, seq: Sequence) -> None:
    if fut.done():
        return
    if seq.finish_reason == "error":
        fut.set_exception(RuntimeError("engine failed"))
    else:
        fut.set_result(seq)


def _set(fut: asyncio.Future, v) -> None:
    if not fut.done():
        fut.set_result(v)


def _fail(fut: asyncio.Future, e: BaseException) -> None:
    if not fut.done():
        fut.set_exception(e)
