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

import asyncio
import logging
import os
import time
import uuid
from typing import Any, Dict, List, Optional

from src.engine.async_engine import AsyncLLMEngine
from src.engine.sequence import Sequence
from src.parallel.kv_transfer import ExportSlot, KVPacket, packet_from_wire, packet_meta, packet_to_wire, ship
from src.preproc import SamplingParams
from src.rpc import RPCClient

logger = logging.getLogger(__name__)


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
        dst = self.decode.engine.device
        if dst.type == "cuda" and pseq.kv_export.is_cuda:  # peer copy on a transfer stream: no host sync
            kv, ready = ship(pseq.kv_export, dst, getattr(pseq, "kv_export_ready", None))
        else:  # a host hop waits for the gather: off the event-loop thread
            kv, ready = await asyncio.to_thread(ship, pseq.kv_export, dst, getattr(pseq, "kv_export_ready", None))
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
    """Prefill worker side of a cross-process pair: sends the packet to a decode worker
    (``op: kv_import``) and returns that worker's reply. On one node the KV payload goes by DMA into
    the decode worker's IPC landing zone (``kv_channel`` once, ``kv_reserve`` per packet; xGMI between
    two GPUs) and only the metadata crosses the socket; anywhere else — or if the zone is full — the
    payload rides the RPC frame as bytes."""

    def __init__(self, address: str, model: str, timeout: float = 600.0, use_ipc: bool = True,
                 reserve_wait_s: float = 30.0):
        self.address = address
        self.reserve_wait_s = reserve_wait_s
        self.model = model
        self.rpc = RPCClient(max_idle_per_host=64, codec=b"M")  # msgpack: raw KV bytes, no base64
        self.timeout = timeout
        self.use_ipc = use_ipc
        self._ipc = None
        self._ipc_lock = asyncio.Lock()
        self.ipc_packets = 0
        self.direct_packets = 0   # gathered by the prefill engine straight into a reserved slot
        self.staged_packets = 0   # gathered locally, then copied into a slot (zone full at submit / deadline)
        self.wire_packets = 0
        self._tasks: set = set()  # background releases: held here (the loop keeps only weak references)
        self.slot_offsets: List[int] = []  # landing-zone offset of every direct packet (slot reuse, tests)

    # seconds kept between the local deadline of a direct export and the decode worker's reservation TTL
    DEADLINE_MARGIN_S = 5.0

    def _spawn(self, coro) -> None:
        t = asyncio.ensure_future(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    @property
    def kv_path(self) -> str:
        """How packets have travelled so far: direct / staged / wire (or mixed, e.g. "direct+staged")."""
        parts = [n for n, c in (("direct", self.direct_packets), ("staged", self.staged_packets),
                                ("wire", self.wire_packets)) if c]
        return "+".join(parts) or "none"

    def stats(self) -> Dict[str, Any]:
        return {"kv_path": self.kv_path, "direct_packets": self.direct_packets, "staged_packets": self.staged_packets,
                "wire_packets": self.wire_packets, "ipc": self._ipc is not None, "decode_worker": self.address}

    async def _channel(self, device):
        if self._ipc is not None or not self.use_ipc or device.type != "cuda":
            return self._ipc
        async with self._ipc_lock:  # concurrent first sends: map the zone once
            return await self._open_channel(device)

    async def _open_channel(self, device):
        if self._ipc is None and self.use_ipc and device.type == "cuda":
            try:
                rep = await self.rpc.call(self.address, {"op": "kv_channel", "model": self.model}, self.timeout)
                if rep.get("success") and rep.get("pid") == os.getpid():
                    self.use_ipc = False  # same process: a handle cannot be opened by its own exporter
                elif rep.get("success"):
                    from src.parallel.kv_transfer import IPCSender

                    self._ipc = IPCSender(rep.get("handles") or rep["handle"], rep.get("seg_bytes", rep["capacity"]),
                                          device)
                    logger.info("KV IPC channel to %s mapped (%d MiB landing zone)", self.address,
                                rep["capacity"] >> 20)
                else:
                    self.use_ipc = False
            except Exception as e:  # different node / no IPC: bytes over the socket from now on
                # loud: on one node this is a misconfiguration (e.g. the decode GPU not visible to this process)
                logger.warning("KV IPC channel to %s unavailable (%s): prompt KV will travel as BYTES over the RPC "
                               "socket (kv_path 'wire')", self.address, e)
                self.use_ipc = False
        return self._ipc

    async def reserve(self, device, shape: List[int], wait_s: Optional[float] = None) -> Optional[Dict[str, Any]]:
        """Reserve a landing-zone slot for a packet of ``shape``: returns ``{"offset", "gen", "dst", "ttl_s"}``
        (``dst`` a bf16 view of the slot for the prefill engine's gather to write into), or None (no IPC
        channel / zone full). ``wait_s``: how long the decode worker may wait for space (default: none)."""
        ch = await self._channel(device)
        if ch is None:
            return None
        nbytes = 2
        for d in shape:
            nbytes *= int(d)
        rep = await self.rpc.call(self.address, {"op": "kv_reserve", "model": self.model, "nbytes": nbytes,
                                                 "wait_s": wait_s or 0.0}, self.timeout)
        if not rep.get("success"):
            return None
        try:
            dst = ch.dst(rep["offset"], shape)
        except ValueError:
            await self._release(rep["offset"], rep.get("gen"))
            return None
        return {"offset": rep["offset"], "gen": rep.get("gen"), "dst": dst, "ttl_s": rep.get("ttl_s", 120.0)}

    async def reserve_export(self, device, shape: List[int]) -> Optional[ExportSlot]:
        """A slot for the prefill engine to gather into, reserved BEFORE the prompt runs and without waiting
        (a full zone must not keep prompts out of the prefill queue: they take the staged path instead). The
        slot's local deadline is taken before the RPC, so it ends before the decode worker's TTL can."""
        t0 = time.monotonic()
        res = await self.reserve(device, shape)
        if res is None:
            return None
        return ExportSlot(res, t0 + float(res["ttl_s"]) - self.DEADLINE_MARGIN_S)

    def revoke(self, slot: ExportSlot) -> None:
        """Give an export slot back (cancelled request, stop token, deadline passed): at once when no gather
        was queued into it, else once that gather's event has completed — a later owner of the slot is never
        overwritten."""
        st, ev = slot.revoke()
        off, gen = slot.res["offset"], slot.res["gen"]
        if st == "taken" and ev is None:  # an overlapped export still queueing its layer groups
            self._spawn(self._release_after_slot_event(slot))
        elif st == "taken" and not ev.query():
            self._spawn(self._release_after_copy(off, gen, ev))
        else:
            self._spawn(self._release(off, gen))

    async def send_reserved(self, packet: KVPacket, slot: Dict[str, Any]) -> Dict[str, Any]:
        """The packet's KV was gathered straight into ``slot`` (see :meth:`reserve`): wait for that gather
        (its event, polled) and hand the slot over with ONE kv_import. If that fails before the decode
        worker owns the slot, the slot is released — after the gather has finished writing it."""
        off, gen = slot["offset"], slot["gen"]
        imported = False
        self.slot_offsets.append(off)
        try:
            await self._ipc.wait_ready(packet.ready)
            wire = dict(packet_meta(packet), ipc={"offset": off, "gen": gen})
            self.ipc_packets += 1
            self.direct_packets += 1
            imported = True
            return await self.rpc.call(self.address, {"op": "kv_import", "model": self.model, "packet": wire},
                                       self.timeout)
        except BaseException:
            if not imported:
                await self.abandon(slot, packet.ready)
            raise

    async def abandon(self, slot: Dict[str, Any], ready=None) -> None:
        """Give a reserved slot back (the prompt failed or was cancelled): once ``ready`` (the gather into
        it, if one was issued) has completed, so no later owner of the slot is overwritten."""
        if ready is not None and not ready.query():
            self._spawn(self._release_after_copy(slot["offset"], slot["gen"], ready))
        else:
            await self._release(slot["offset"], slot["gen"])

    async def send(self, packet: KVPacket) -> Dict[str, Any]:
        ch = await self._channel(packet.kv.device)
        if ch is not None:
            # the decode worker waits (briefly) for a slot to come back rather than refuse: slots return as
            # soon as its engine has scattered them, and the byte path is far slower than waiting
            rep = await self.rpc.call(self.address, {"op": "kv_reserve", "model": self.model,
                                                     "nbytes": packet.nbytes, "wait_s": self.reserve_wait_s},
                                      self.timeout)
            if rep.get("success"):
                self.staged_packets += 1
                off, gen = rep["offset"], rep.get("gen")
                imported = False
                issued: Dict[str, Any] = {}
                try:
                    # the copy runs on a transfer stream after the prefill engine's gather; the event loop
                    # only polls its completion event (no synchronize on this thread)
                    await ch.write_async(off, packet.kv, packet.ready, issued=issued)
                    wire = dict(packet_meta(packet), ipc={"offset": off, "gen": gen})
                    self.ipc_packets += 1
                    imported = True  # from here the decode worker owns the slot (released after its scatter)
                    return await self.rpc.call(self.address, {"op": "kv_import", "model": self.model,
                                                              "packet": wire}, self.timeout)
                except BaseException:
                    if not imported:  # the slot would leak: hand it back (best effort; it also expires)
                        ev = issued.get("event")
                        if ev is not None and not ev.query():
                            # cancelled while the copy still writes into the slot: release it only once the
                            # copy has finished, or another sender could get the slot and be overwritten
                            self._spawn(self._release_after_copy(off, gen, ev))
                        else:
                            await self._release(off, gen)
                    raise
        self.wire_packets += 1
        # device -> host copy of the payload: off the event-loop thread
        msg = {"op": "kv_import", "model": self.model, "packet": await asyncio.to_thread(packet_to_wire, packet)}
        return await self.rpc.call(self.address, msg, self.timeout)


    async def _release(self, off: int, gen) -> None:
        try:
            await self.rpc.call(self.address, {"op": "kv_release", "model": self.model, "offset": off, "gen": gen},
                                30.0)
        except Exception:
            logger.warning("kv_release of slot %d on %s failed", off, self.address)

    async def _release_after_slot_event(self, slot: ExportSlot, poll_s: float = 1e-3, limit_s: float = 60.0) -> None:
        t0 = time.monotonic()
        while slot.event is None:
            if time.monotonic() - t0 > limit_s:  # the engine never finished the export: leave it to the TTL
                logger.warning("export into slot %d never completed; slot left to expire", slot.res["offset"])
                return
            await asyncio.sleep(poll_s)
        await self._release_after_copy(slot.res["offset"], slot.res["gen"], slot.event)

    async def _release_after_copy(self, off: int, gen, ev, poll_s: float = 2e-4, limit_s: float = 60.0) -> None:
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > limit_s:  # never completes: leave the slot to the reservation TTL
                logger.warning("KV copy into slot %d never completed; slot left to expire", off)
                return
            await asyncio.sleep(poll_s)
        await self._release(off, gen)


def sampling_to_dict(sp: SamplingParams) -> Dict[str, Any]:
    return {"max_tokens": sp.max_tokens, "temperature": sp.temperature, "top_k": sp.top_k, "top_p": sp.top_p,
            "seed": sp.seed, "ignore_eos": sp.ignore_eos, "stop_token_ids": list(sp.stop_token_ids)}


def packet_for_import(d: Dict[str, Any], device) -> KVPacket:
    return packet_from_wire(d, device)
