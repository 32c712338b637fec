"""
Wire format for the coordinator/worker control plane.

The reference protocol is "write one JSON object, read until EOF, one request
per connection" with a single ``reader.read(4096)`` on the server
(`/root/reference/src/worker.py:93,116-124`) — anything over 4 KiB breaks.
`README.md:101` promises length-prefixed frames; this module implements them:

    frame := u32_be(len(body)) || body
    body  := codec_byte || payload       codec_byte ∈ {b'J' json, b'M' msgpack, b'P' pickle}

Frames allow many request/response pairs on one persistent connection.
Legacy clients are still served: a connection whose first byte is ``{`` is
read as one unframed JSON document and answered unframed (then closed).
Pickle is never accepted from the network unless explicitly enabled.
"""

from __future__ import annotations

import asyncio
import json
import pickle
import re
import struct
from typing import Any, Optional, Tuple

try:  # msgpack is in the image's wheelhouse; JSON is the always-available default
    import msgpack  # type: ignore
except Exception:  # pragma: no cover
    msgpack = None

MAX_FRAME = 1 << 30  # 1 GiB; a legacy '{' first byte can never be a valid length prefix
_HDR = struct.Struct(">I")

CODEC_JSON = b"J"
CODEC_MSGPACK = b"M"
CODEC_PICKLE = b"P"


class ProtocolError(Exception):
    pass


def serialize(obj: Any, codec: bytes = CODEC_JSON) -> bytes:
    """Encode ``obj`` into a frame body (codec byte + payload)."""
    if codec == CODEC_JSON:
        return codec + json.dumps(obj, separators=(",", ":")).encode()
    if codec == CODEC_MSGPACK:
        if msgpack is None:
            raise ProtocolError("msgpack unavailable")
        return codec + msgpack.packb(obj, use_bin_type=True)
    if codec == CODEC_PICKLE:
        return codec + pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    raise ProtocolError(f"unknown codec {codec!r}")


def deserialize(body: bytes, allow_pickle: bool = False) -> Any:
    """Decode a frame body produced by :func:`serialize`."""
    if not body:
        raise ProtocolError("empty frame")
    codec, payload = body[:1], body[1:]
    if codec == CODEC_JSON:
        return json.loads(payload)
    if codec == CODEC_MSGPACK:
        if msgpack is None:
            raise ProtocolError("msgpack unavailable")
        return msgpack.unpackb(payload, raw=False, strict_map_key=False)
    if codec == CODEC_PICKLE:
        if not allow_pickle:
            raise ProtocolError("pickle frames are disabled")
        return pickle.loads(payload)
    raise ProtocolError(f"unknown codec {codec!r}")


def pack_frame(obj: Any, codec: bytes = CODEC_JSON) -> bytes:
    body = serialize(obj, codec)
    if len(body) > MAX_FRAME:
        raise ProtocolError("frame too large")
    return _HDR.pack(len(body)) + body


async def read_frame(reader: asyncio.StreamReader, allow_pickle: bool = False) -> Tuple[Any, bytes]:
    """Read one framed message. Returns ``(obj, codec)``; raises
    ``asyncio.IncompleteReadError`` on a clean EOF before the header."""
    hdr = await reader.readexactly(4)
    (n,) = _HDR.unpack(hdr)
    if n == 0 or n > MAX_FRAME:
        raise ProtocolError(f"bad frame length {n}")
    body = await reader.readexactly(n)
    return deserialize(body, allow_pickle=allow_pickle), body[:1]


async def write_frame(writer: asyncio.StreamWriter, obj: Any, codec: bytes = CODEC_JSON) -> None:
    writer.write(pack_frame(obj, codec))
    await writer.drain()


_STRUCT = re.compile(rb'["\\{}\[\]]')


class _JsonObjectEnd:
    """Incremental scanner for the end of one top-level JSON object: tracks brace depth outside strings
    (with escapes), so each byte is looked at once however the document is chunked."""

    __slots__ = ("depth", "in_str", "esc")

    def __init__(self) -> None:
        self.depth = 0
        self.in_str = False
        self.esc = False

    def feed(self, data: bytes, base: int) -> int:
        """Scan ``data`` (at offset ``base`` of the stream); return the stream offset one past the object's
        closing brace, or -1 if it has not closed yet. Only the structural bytes are visited."""
        depth, in_str, esc = self.depth, self.in_str, self.esc
        # position of the previous structural byte (a backslash escapes only the byte right after it; one
        # that ended the previous chunk escapes byte 0 of this one)
        last = -1 if esc else -2
        for m in _STRUCT.finditer(data):
            i = m.start()
            c = data[i]
            if esc and i == last + 1:
                esc = False
                last = i
                continue
            esc = False
            last = i
            if in_str:
                if c == 0x5C:  # backslash
                    esc = True
                elif c == 0x22:  # quote
                    in_str = False
            elif c == 0x22:
                in_str = True
            elif c == 0x7B or c == 0x5B:  # { [
                depth += 1
            elif c == 0x7D or c == 0x5D:  # } ]
                depth -= 1
                if depth == 0:
                    self.depth, self.in_str, self.esc = depth, in_str, esc
                    return base + i + 1
        if esc and last != len(data) - 1:
            esc = False  # the escaped byte was an ordinary character
        self.depth, self.in_str, self.esc = depth, in_str, esc
        return -1


async def read_legacy_json(reader: asyncio.StreamReader, first: bytes, limit: int = MAX_FRAME) -> Any:
    """Read an unframed JSON document that started with ``first``: accumulate chunks until the top-level
    object closes (one linear scan), then decode it once; at EOF decode what arrived (raises the real
    error if it is incomplete)."""
    buf = bytearray(first)
    scan = _JsonObjectEnd()
    end = scan.feed(first, 0)
    while end < 0:
        chunk = await reader.read(65536)
        if not chunk:
            return json.loads(buf.decode())
        base = len(buf)
        buf += chunk
        if len(buf) > limit:
            raise ProtocolError("legacy request too large")
        end = scan.feed(chunk, base)
    return json.loads(bytes(buf[:end]).decode())


async def read_message(reader: asyncio.StreamReader, allow_pickle: bool = False) -> Tuple[Optional[Any], str, bytes]:
    """Server side: read one request in either format.

    Returns ``(obj, mode, codec)`` with ``mode`` ``"framed"`` or ``"legacy"``;
    ``(None, "eof", b"")`` when the peer closed without sending anything
    (a TCP-connect health probe).
    """
    first = await reader.read(1)
    if not first:
        return None, "eof", b""
    # Only '{' marks a legacy request: the reference client always sends json.dumps(dict). Whitespace
    # bytes are NOT accepted as a legacy start because 0x09/0x0A/0x0D/0x20 are valid high bytes of a
    # frame length (144-176 MiB, 208-224 MiB, 512-528 MiB: e.g. a 4K-token Llama-3-8B kv_import).
    # 0x7B << 24 exceeds MAX_FRAME, so '{' can never start a valid frame header.
    if first == b"{":
        return await read_legacy_json(reader, first), "legacy", CODEC_JSON
    rest = await reader.readexactly(3)
    (n,) = _HDR.unpack(first + rest)
    if n == 0 or n > MAX_FRAME:
        raise ProtocolError(f"bad frame length {n}")
    body = await reader.readexactly(n)
    return deserialize(body, allow_pickle=allow_pickle), "framed", body[:1]
