"""
Disaggregated serving: prefill on one engine/GPU, decode on another
(BASELINE config 3; the reference only names "disaggregated inference",
`/root/reference/README.md:15`).

Prefill-heavy and decode-heavy phases want different batch shapes: the
prefill GPU runs large ragged batches at high MFMA utilisation while the
decode GPU keeps a full continuous batch streaming weights from HBM. The
prompt KV moves once, as packed blocks (see :mod:`src.parallel.kv_transfer`).

:class:`DisaggregatedServer` pairs two :class:`AsyncLLMEngine` instances in
one process (GPU→GPU peer copy over xGMI, or the same GPU for a 1-GPU box);
:class:`RemoteDecodeLink` ships packets to a decode *worker* over the
control-plane RPC (``op: kv_import``).
"""

from __future__ import annotations

import time
import uuid
from typing import Any, Dict, List, Optional

from src.engine.async_engine import AsyncLLMEngine
from src.engine.sequence import Sequence
from src.parallel.kv_transfer import KVPacket, packet_from_wire, packet_to_wire, ship
from src.preproc import SamplingParams
from src.rpc import RPCClient


class DisaggregatedServer:
    def __init__(self, prefill: AsyncLLMEngine, decode: AsyncLLMEngine):
        if prefill.engine.cfg.block_size != decode.engine.cfg.block_size:
            raise ValueError("prefill and decode engines need the same KV block size")
        self.prefill = prefill
        self.decode = decode
        self.transfers = 0
        self.bytes_moved = 0
        self.transfer_s = 0.0

    def start(self) -> None:
        self.prefill.start()
        self.decode.start()

    def stop(self) -> None:
        self.prefill.stop()
        self.decode.stop()

    async def generate(self, prompt_ids: List[int], sampling: SamplingParams,
                       request_id: Optional[str] = None) -> Sequence:
        rid = request_id or uuid.uuid4().hex
        pseq = await self.prefill.submit(rid, prompt_ids, sampling, user_data={"export_kv": True})
        if pseq.finish_reason == "stop" or sampling.max_tokens <= 1:
            pseq.sampling = sampling
            return pseq
        t0 = time.perf_counter()
        kv, ready = ship(pseq.kv_export, self.decode.engine.device, getattr(pseq, "kv_export_ready", None))
        self.transfer_s += time.perf_counter() - t0   # issue time: the copy itself is asynchronous
        self.transfers += 1
        self.bytes_moved += kv.numel() * kv.element_size()
        packet = KVPacket(rid, list(prompt_ids), pseq.output_ids[0], kv, self.prefill.engine.cfg.block_size,
                          ttft_ms=pseq.ttft_ms(), ready=ready)
        pseq.kv_export = None
        return await self.decode.submit(rid, [], sampling, user_data={"import_packet": packet})

    def stats(self) -> Dict[str, Any]:
        return {"transfers": self.transfers, "bytes_moved": self.bytes_moved,
                "transfer_ms_avg": 1e3 * self.transfer_s / max(1, self.transfers),
                "prefill": self.prefill.stats(), "decode": self.decode.stats()}


class RemoteDecodeLink:
    """Prefill worker side of a cross-process pair: sends the packet to a
    decode worker (``op: kv_import``) and returns that worker's reply."""

    def __init__(self, address: str, model: str, timeout: float = 600.0):
        self.address = address
        self.model = model
        self.rpc = RPCClient(max_idle_per_host=64, codec=b"M")  # msgpack: raw KV bytes, no base64
        self.timeout = timeout

    async def send(self, packet: KVPacket) -> Dict[str, Any]:
        msg = {"op": "kv_import", "model": self.model, "packet": packet_to_wire(packet)}
        return await self.rpc.call(self.address, msg, self.timeout)


def sampling_to_dict(sp: SamplingParams) -> Dict[str, Any]:
    return {"max_tokens": sp.max_tokens, "temperature": sp.temperature, "top_k": sp.top_k, "top_p": sp.top_p,
            "seed": sp.seed, "ignore_eos": sp.ignore_eos, "stop_token_ids": list(sp.stop_token_ids)}


def packet_for_import(d: Dict[str, Any], device) -> KVPacket:
    return packet_from_wire(d, device)
