"""
Shared helpers (`/root/reference/README.md:36,100-102` promised a ``utils.py``
with ``serialize``/``deserialize`` over length-prefixed frames and a simple
tracer; neither exists in the reference).
"""

import logging
import os

from .framing import (  # noqa: F401
    CODEC_JSON,
    CODEC_MSGPACK,
    CODEC_PICKLE,
    ProtocolError,
    deserialize,
    pack_frame,
    read_frame,
    read_message,
    serialize,
    write_frame,
)
from .tracing import GLOBAL_TRACER, Trace, Tracer, new_request_id, percentile  # noqa: F401


def setup_logging(level: str = None) -> None:
    """Configure logging once for CLIs (library modules never call basicConfig,
    unlike the reference which does so at import time in four modules)."""
    lvl = (level or os.environ.get("DIE_LOG_LEVEL", "INFO")).upper()
    logging.basicConfig(level=getattr(logging, lvl, logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")


def parse_address(addr: str):
    host, _, port = addr.rpartition(":")
    if not host:
        raise ValueError(f"address must be host:port, got {addr!r}")
    return host, int(port)
