"""
Client for the coordinator / worker RPC API (the reference promises
``examples/example_client.py`` at `README.md:38`; this is its library half).
"""

from __future__ import annotations

import asyncio
import json
from typing import Any, Dict, Optional

from src.rpc import RPCClient
from src.utils import parse_address
from src.utils.framing import CODEC_JSON, CODEC_MSGPACK, msgpack


class InferenceClient:
    """Framed RPC client. Frames are msgpack when it is importable (servers answer in the request's codec;
    JSON encoding of every reply was the largest single cost of the coordinator's request path), JSON
    otherwise or with ``codec="json"``."""

    def __init__(self, address: str, timeout: float = 600.0, codec: str = "msgpack"):
        self.address = address
        self.timeout = timeout
        use_mp = codec == "msgpack" and msgpack is not None
        self._rpc = RPCClient(max_idle_per_host=1024, codec=CODEC_MSGPACK if use_mp else CODEC_JSON)

    async def infer(self, model: str, inputs: Any, version: Optional[str] = None,
                    request_key: Optional[str] = None, cache: bool = True, **extra) -> Dict[str, Any]:
        msg: Dict[str, Any] = {"op": "infer", "model": model, "inputs": inputs, "cache": cache}
        if version:
            msg["version"] = version
        if request_key:
            msg["request_key"] = request_key
        msg.update(extra)
        return await self._rpc.call(self.address, msg, self.timeout)

    async def infer_stream(self, model: str, inputs: Any, version: Optional[str] = None,
                           request_key: Optional[str] = None, **extra):
        """Streamed generation: yields ``{"delta_token_ids": [...], "done": False}`` frames as tokens are
        produced, then the final response (``"done": True``, same shape as :meth:`infer`'s reply)."""
        inputs = dict(inputs, stream=True)
        msg: Dict[str, Any] = {"op": "infer", "model": model, "inputs": inputs, "cache": False}
        if version:
            msg["version"] = version
        if request_key:
            msg["request_key"] = request_key
        msg.update(extra)
        async for frame in self._rpc.stream(self.address, msg, self.timeout):
            yield frame

    async def abort(self, model: str, request_id: str) -> Dict[str, Any]:
        """Abort a running request on a worker (frees its batch slot and KV blocks)."""
        return await self.call({"op": "abort", "model": model, "request_id": request_id})

    async def submit(self, model: str, inputs: Any, **kw) -> str:
        rep = await self._rpc.call(self.address, dict({"op": "submit", "model": model, "inputs": inputs}, **kw),
                                   self.timeout)
        if not rep.get("success"):
            raise RuntimeError(rep.get("error"))
        return rep["request_id"]

    async def result(self, request_id: str, poll_s: float = 0.01, timeout: Optional[float] = None) -> Dict[str, Any]:
        loop = asyncio.get_running_loop()
        deadline = loop.time() + (timeout or self.timeout)
        while True:
            rep = await self._rpc.call(self.address, {"op": "result", "request_id": request_id}, self.timeout)
            if rep.get("status") != "pending":
                return rep
            if loop.time() > deadline:
                raise asyncio.TimeoutError(request_id)
            await asyncio.sleep(poll_s)

    async def call(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        return await self._rpc.call(self.address, msg, self.timeout)

    async def stats(self) -> Dict[str, Any]:
        return await self.call({"op": "stats"})

    def close(self) -> None:
        self._rpc.close()


async def legacy_request(address: str, msg: Dict[str, Any], timeout: float = 30.0) -> Dict[str, Any]:
    """The reference wire format: write raw JSON, read until the server closes."""
    host, port = parse_address(address)
    r, w = await asyncio.wait_for(asyncio.open_connection(host, port), timeout)
    w.write(json.dumps(msg).encode())
    await w.drain()
    data = await asyncio.wait_for(r.read(), timeout)
    w.close()
    return json.loads(data.decode())
