"""
Framed-JSON RPC client with persistent, pooled connections.

The reference opens one TCP connection per request and closes it after the
reply (`/root/reference/src/worker.py:116-124`); health probes are bare TCP
connects (`src/router.py:287-292`, `src/load_balancer.py:326-331`). Here a
client keeps a small pool of framed connections per worker address and
multiplexes sequential requests over them; probes are real ``{"op":"health"}``
RPCs so a worker can tell a probe from a request.
"""

from __future__ import annotations

import asyncio
import contextlib
import time
from collections import defaultdict
from typing import Any, Dict, List, Optional, Tuple

from src.utils import CODEC_JSON, parse_address, read_frame, pack_frame
from src.utils.frameserver import FrameClientProtocol


class RPCError(Exception):
    pass


class _Conn:
    __slots__ = ("reader", "writer")

    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        self.reader = reader
        self.writer = writer

    def close(self) -> None:
        with contextlib.suppress(Exception):
            self.writer.close()


class RPCClient:
    def __init__(self, max_idle_per_host: int = 64, codec: bytes = CODEC_JSON):
        self.max_idle = max_idle_per_host
        self.codec = codec
        self._idle: Dict[str, List[_Conn]] = defaultdict(list)

    async def _open(self, address: str, timeout: float) -> _Conn:
        host, port = parse_address(address)
        r, w = await asyncio.wait_for(asyncio.open_connection(host, port, limit=1 << 26), timeout)
        return _Conn(r, w)

    async def _open_proto(self, address: str, timeout: float) -> FrameClientProtocol:
        host, port = parse_address(address)
        loop = asyncio.get_running_loop()
        _, proto = await asyncio.wait_for(loop.create_connection(FrameClientProtocol, host, port), timeout)
        return proto

    async def call(self, address: str, msg: Any, timeout: Optional[float] = 600.0) -> Any:
        """Send one framed request and await its framed reply (a pooled protocol-level connection: the reply
        frame is cut out of the receive buffer by the connection's callback, no reader task per call)."""
        pool = self._idle[address]
        conn = None
        while pool and conn is None:
            c = pool.pop()
            conn = None if c.closed else c
        fresh = conn is None
        if conn is None:
            conn = await self._open_proto(address, timeout or 30.0)
        # the reply timeout aborts the connection from a timer instead of wrapping the read in
        # asyncio.wait_for (a task + a timer per call on Python 3.10: the RPC hot path's largest cost)
        timer, expired = None, []
        if timeout:
            def _expire(t=conn.transport):
                expired.append(True)
                t.abort()
            timer = asyncio.get_running_loop().call_later(timeout, _expire)
        try:
            reply = await conn.request(pack_frame(msg, self.codec))
        except (ConnectionError, OSError) as e:
            conn.close()
            if expired:
                raise asyncio.TimeoutError(f"rpc to {address}: no reply within {timeout} s") from e
            if not fresh:
                # A pooled connection may have been closed by the peer while idle: retry once fresh.
                if timer is not None:
                    timer.cancel()
                return await self.call(address, msg, timeout)
            raise RPCError(f"rpc to {address} failed: {e}") from e
        except BaseException:
            conn.close()
            raise
        finally:
            if timer is not None:
                timer.cancel()
        if len(pool) < self.max_idle and not conn.closed:
            pool.append(conn)
        else:
            conn.close()
        return reply

    async def stream(self, address: str, msg: Any, timeout: Optional[float] = 600.0):
        """Send one request whose reply is streamed: yields every frame; intermediate frames carry
        ``"done": False``, the last one does not. Uses a dedicated connection (closed at the end), so a
        consumer that stops early simply drops the connection and the server aborts the request."""
        conn = await self._open(address, timeout or 30.0)
        try:
            conn.writer.write(pack_frame(msg, self.codec))
            await conn.writer.drain()
            while True:
                frame, _ = await asyncio.wait_for(read_frame(conn.reader), timeout)
                yield frame
                if not (isinstance(frame, dict) and frame.get("done") is False):
                    return
        except (ConnectionError, asyncio.IncompleteReadError, OSError) as e:
            raise RPCError(f"stream from {address} failed: {e}") from e
        finally:
            conn.close()

    async def probe(self, address: str, timeout: float = 2.0,
                    msg: Optional[Dict[str, Any]] = None) -> Tuple[bool, float, Optional[Dict[str, Any]]]:
        """Health RPC on a dedicated short-lived connection. Returns
        ``(ok, latency_s, reply)``; the latency is the probe's own round trip
        and is kept apart from request latency statistics."""
        t0 = time.perf_counter()
        conn = None
        try:
            conn = await self._open(address, timeout)
            conn.writer.write(pack_frame(msg or {"op": "health"}, CODEC_JSON))
            await conn.writer.drain()
            reply, _ = await asyncio.wait_for(read_frame(conn.reader), timeout)
            ok = bool(reply.get("success", False)) if isinstance(reply, dict) else False
            return ok, time.perf_counter() - t0, reply
        except (asyncio.TimeoutError, OSError, ConnectionError, asyncio.IncompleteReadError, ValueError):
            return False, time.perf_counter() - t0, None
        finally:
            if conn is not None:
                conn.close()

    def close(self) -> None:
        for conns in self._idle.values():
            for c in conns:
                c.close()
        self._idle.clear()


async def tcp_connect_probe(address: str, timeout: float) -> Tuple[bool, float]:
    """The reference's probe: can we open a TCP connection?"""
    t0 = time.perf_counter()
    try:
        host, port = parse_address(address)
        _, w = await asyncio.wait_for(asyncio.open_connection(host, port), timeout)
        w.close()
        with contextlib.suppress(Exception):
            await w.wait_closed()
        return True, time.perf_counter() - t0
    except (asyncio.TimeoutError, OSError, ValueError):
        return False, time.perf_counter() - t0
