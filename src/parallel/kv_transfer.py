"""
KV-block transfer for disaggregated prefill → decode (BASELINE config 3).

A prefill worker computes a prompt's KV into its paged pool, packs the
sequence's blocks (every layer, K and V) into one contiguous staging tensor
with the ``move_blocks`` HIP kernel, and ships it to the decode worker's GPU:

* same process, other GPU  → ``tensor.to(dst)`` = ``hipMemcpyPeerAsync`` over
  xGMI (SDMA engines; compute keeps running);
* other process, same node → a device-to-device copy into the decode worker's
  IPC-mapped landing zone (:class:`IPCSender` / :class:`IPCLandingZone`), or
  RCCL point-to-point between ranks of one group (:class:`RCCLChannel`);
* anywhere else            → framed bytes over the control-plane TCP socket
  (:func:`packet_to_wire` / :func:`packet_from_wire`), the CPU fallback.

The decode worker allocates fresh blocks, scatters the staging tensor into
them (``move_blocks`` again) and resumes the sequence as a running decode —
no prompt recompute. For Llama-3-8B a 512-token prompt is 64 MiB of KV.
"""

from __future__ import annotations

from dataclasses import dataclass, field
import threading
import time
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from src import ops


@dataclass
class KVPacket:
    request_id: str
    prompt_ids: List[int]
    first_token: int
    kv: torch.Tensor                 # [n_blocks, planes, slab] (bf16)
    block_size: int
    sampling: Dict[str, Any] = field(default_factory=dict)
    ttft_ms: Optional[float] = None
    ready: Any = None                # HIP event: kv is complete on its device (None = already complete)
    # called by the importing engine thread with an event recorded behind its scatter (the kv buffer
    # may be reused once that event completes): frees an IPC landing-zone slot without a host sync
    on_imported: Optional[Callable[[Any], None]] = None

    @property
    def nbytes(self) -> int:
        return self.kv.numel() * self.kv.element_size()


class ExportSlot:
    """A decode worker's landing-zone slot, reserved before a prompt runs, that the prefill engine may gather
    the prompt's KV straight into — the hand-over between the event-loop thread (which reserved it and may
    revoke it) and the engine thread (which takes it when the prompt finishes). Thread-safe.

    The decode worker expires an un-imported reservation after its TTL and may then give the offset to another
    sender; a gather issued after that would overwrite the new owner's KV. So the slot carries a local
    ``deadline`` (reserve time on THIS side, taken before the reserve RPC, + the decode worker's TTL − a
    margin): past it the engine gathers into a local staging tensor instead, and the packet takes the staged
    path. States: ``open`` → ``taken`` (a gather into it was queued; ``event`` marks its completion) or
    ``expired`` (the deadline passed first) or ``revoked`` (the request was cancelled first)."""

    def __init__(self, reservation: Dict[str, Any], deadline: float):
        self.res = reservation            # {"offset", "gen", "dst"} from RemoteDecodeLink.reserve
        self.deadline = deadline          # time.monotonic() on this process
        self.state = "open"
        self.event = None
        self._lock = threading.Lock()

    def gather(self, fn: Callable[[Optional[torch.Tensor]], Any]):
        """Engine thread: ``fn(dst)`` queues the gather (into the slot, or into a fresh staging tensor when
        ``dst`` is None) and returns ``(tensor, event)``. The state changes under the lock, together with
        the issue, so a concurrent :meth:`revoke` sees either no gather or a gather with its event."""
        with self._lock:
            if self.state == "open" and time.monotonic() < self.deadline:
                out, ev = fn(self.res["dst"])
                self.state, self.event = "taken", ev
                return out, ev
            if self.state == "open":
                self.state = "expired"
        return fn(None)

    def set_event(self, ev) -> None:
        """Engine thread: the completion event of a gather queued in pieces (overlapped export)."""
        with self._lock:
            self.event = ev

    def revoke(self):
        """Event-loop thread: no gather may start after this. Returns ``(state, event)`` as they were: the
        slot is free to release at once unless a gather was queued (``taken``: release after ``event``)."""
        with self._lock:
            st = self.state
            if st == "open":
                self.state = "revoked"
            return st, self.event


_EXPORT_STREAMS: Dict[Any, Any] = {}


class LayerGroupExporter:
    """Overlapped export of the prompts that finish in a prefill step (disaggregated prefill → decode): as soon as
    the forward has queued the KV writes of each group of ``group`` layers, the gather of those layers' planes
    (every finishing prompt's blocks, each into its own packet: a decode worker's landing-zone slot over xGMI, or
    a staging tensor) is queued on a separate export stream behind an event — the copies run while the
    remaining layers compute, and only the last group's copy is left after the forward. ``finish()`` queues
    whatever is left (a forward without layer callbacks exports everything there), returns the completion event
    and makes the compute stream wait for it, so no later kernel can reuse the exported blocks before they
    were read."""

    def __init__(self, pool_planes: torch.Tensor, num_layers: int, targets: List[Any], group: int = 4):
        self.pool = pool_planes
        self.device = pool_planes.device
        self.planes = pool_planes.shape[0]
        self.per_layer = self.planes // num_layers
        self.num_layers = num_layers
        self.group = max(1, group)
        self.done = 0
        ids, dst = [], []
        row = self.planes * (pool_planes.numel() // (self.planes * pool_planes.shape[1])) * pool_planes.element_size()
        self.targets = targets                # [(block_ids, packet [nb, planes, slab])], kept alive until finish
        for block_ids, buf in targets:
            base = buf.data_ptr()
            for j, b in enumerate(block_ids):
                ids.append(int(b))
                dst.append(base + j * row)
        self.ids = torch.tensor(ids, dtype=torch.int64, device=self.device)
        self.dst = torch.tensor(dst, dtype=torch.int64, device=self.device)
        s = _EXPORT_STREAMS.get(self.device)
        if s is None:
            s = _EXPORT_STREAMS[self.device] = torch.cuda.Stream(device=self.device)
        self.stream = s

    def on_layer(self, li: int) -> None:
        """Called by the forward once layer ``li``'s KV writes are queued on the current stream."""
        if (li + 1) % self.group == 0 or li + 1 == self.num_layers:
            self._gather_upto((li + 1) * self.per_layer)

    def _gather_upto(self, p1: int) -> None:
        if p1 <= self.done:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            ops.gather_blocks_rows(self.pool, self.ids, self.dst, self.done, p1 - self.done)
        self.done = p1

    def finish(self):
        self._gather_upto(self.planes)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        torch.cuda.current_stream(self.device).wait_event(ev)
        for t in (self.ids, self.dst, *(b for _, b in self.targets)):
            t.record_stream(self.stream)
        return ev


def export_blocks(pool_planes: torch.Tensor, block_ids: List[int], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gather ``block_ids`` of every (layer, K/V) plane into a staging tensor, or into ``out`` (e.g. a
    peer's IPC landing-zone slot: the gather then writes straight over xGMI, no second copy)."""
    ids = torch.tensor(block_ids, dtype=torch.int64, device=pool_planes.device)
    return ops.gather_blocks(pool_planes, ids, buf=out)


def packet_shape(pool_planes: torch.Tensor, n_blocks: int) -> List[int]:
    """[n_blocks, planes, slab] of a packet gathered from ``pool_planes`` ([planes, num_blocks, ...])."""
    planes, nb = pool_planes.shape[0], pool_planes.shape[1]
    return [int(n_blocks), int(planes), int(pool_planes.numel() // (planes * nb))]


def import_blocks(pool_planes: torch.Tensor, block_ids: List[int], buf: torch.Tensor) -> None:
    ids = torch.tensor(block_ids, dtype=torch.int64, device=pool_planes.device)
    if buf.device != pool_planes.device:
        buf = buf.to(pool_planes.device, non_blocking=True)
    ops.scatter_blocks(pool_planes, ids, buf.contiguous())


_XFER_STREAMS: Dict[Any, Any] = {}


def _transfer_stream(device: torch.device):
    s = _XFER_STREAMS.get(device)
    if s is None:
        s = _XFER_STREAMS[device] = torch.cuda.Stream(device=device)
    return s


def ship(buf: torch.Tensor, device, ready=None):
    """Move a staging tensor to ``device`` without a host sync: peer copy
    (hipMemcpyPeerAsync over xGMI) on a dedicated per-device transfer stream that
    first waits for ``ready`` (the prefill engine's gather); returns ``(tensor, event)``
    where the event marks the copy's completion — the decode engine makes its
    stream wait on it before scattering the blocks. Same device: no copy."""
    device = torch.device(device)
    if buf.device == device:
        return buf, ready
    if device.type != "cuda" or buf.device.type != "cuda":
        if ready is not None:
            ready.synchronize()
        return buf.to(device), None
    s = _transfer_stream(device)
    with torch.cuda.stream(s):
        if ready is not None:
            s.wait_event(ready)
        out = buf.to(device, non_blocking=True)
        done = torch.cuda.Event()
        done.record(s)
    buf.record_stream(s)   # the source block may not be reused before the copy has read it
    return out, done


class IPCLandingZone:
    """Decode-worker side of cross-process KV shipping on one node: IPC-shareable device segments (plain
    hipMalloc, so this GPU reads them through its caches) that prefill workers map (hipIpcOpenMemHandle)
    and fill over xGMI — the packed prompt KV never touches host memory or the RPC socket, which then
    carries only the metadata. A prefill worker that reserved its slot before the prompt ran gathers the
    prompt's blocks from its paged pool STRAIGHT into the slot (one pass, no staging copy); the decode
    engine then scatters from the slot into its own pool.

    Lifecycle of a slot (no host synchronisation anywhere):
    ``reserve`` (kv_reserve RPC, first fit) → the sender fills it and tells us (kv_import) → ``claim``
    hands the engine a VIEW of the slot (no clone) → the engine thread scatters it straight into its
    paged pool with ``move_blocks`` and calls ``release_after`` with an event recorded behind the
    scatter → the slot returns to the free list once that event has completed (checked without
    blocking whenever space is reserved). A reservation that is never imported (sender failed, client
    gone) is returned by ``release`` (kv_release RPC) or expires after ``reserve_ttl_s``.

    Offsets are global over the segments (segment s covers [s * seg_bytes, (s + 1) * seg_bytes)); a slot
    never spans two. Each segment stays below 2 GiB: on this ROCm (7.2, dmabuf IPC) hipIpcOpenMemHandle of
    a 2 GiB allocation never returns in the importing process, while 256 MiB..1 GiB open in < 10 ms
    (measured, scripts/repro_ipc_kv.py). The default 4 x 1 GiB holds 64 in-flight 512-token Llama-3-8B
    prompts: a whole bench wave of 32 (with one segment, half the wave waited for the other half's
    scatter)."""

    ALIGN = 1 << 16
    MAX_BYTES = (1 << 31) - (1 << 20)   # per segment
    SEG_BYTES = 1 << 30

    def __init__(self, device, capacity: int = 4 << 30, uncached: bool = False, reserve_ttl_s: float = 120.0,
                 seg_bytes: int = SEG_BYTES):
        from src import _C

        self.device = torch.device(device)
        self.seg_bytes = int(min(seg_bytes, capacity))
        if not 0 < self.seg_bytes <= self.MAX_BYTES or self.seg_bytes % self.ALIGN:
            raise ValueError(f"landing-zone segments of {self.seg_bytes} bytes: must be a multiple of "
                             f"{self.ALIGN} in (0, {self.MAX_BYTES}]")
        nseg = max(1, -(-int(capacity) // self.seg_bytes))
        self.capacity = nseg * self.seg_bytes
        self.ptrs, self.views, self.handles = [], [], []
        with torch.cuda.device(self.device):
            for _ in range(nseg):
                ptr = _C.car_alloc(self.seg_bytes, uncached)
                self.ptrs.append(ptr)
                self.views.append(_C.car_tensor(ptr, self.seg_bytes, self.device.index or 0))
                self.handles.append(_C.car_handle(ptr).hex())
        self.handle = self.handles[0]
        self._init_book(reserve_ttl_s)

    def _init_book(self, reserve_ttl_s: float) -> None:
        """Slot bookkeeping (host only; CPU-testable without a device buffer)."""
        self.reserve_ttl_s = reserve_ttl_s
        if not getattr(self, "seg_bytes", None):
            self.seg_bytes = self.capacity
        self._free: List[List[int]] = [[o, o + self.seg_bytes] for o in range(0, self.capacity, self.seg_bytes)]
        self._used: Dict[int, int] = {}
        # generation of each reservation: a late kv_import / kv_release of an expired reservation whose
        # offset was handed out again must not touch the new owner's slot
        self._gen_of: Dict[int, int] = {}
        self._next_gen = 1
        self._reserved_at: Dict[int, float] = {}   # reserved, not yet imported (expire after the TTL)
        self._pending: List[Any] = []              # (offset, event): released once the scatter has run
        self._lock = threading.Lock()
        self.expired = 0

    def _reap(self) -> None:
        now = time.monotonic()
        with self._lock:
            done, keep = [], []
            for o, e in self._pending:  # query each event once: it may complete between two looks
                (done if e is None or e.query() else keep).append((o, e))
            self._pending = keep
            stale = [o for o, t in self._reserved_at.items() if now - t > self.reserve_ttl_s]
        for o, _ in done:
            self.release(o)
        for o in stale:
            self.expired += 1
            self.release(o)

    def reserve(self, nbytes: int) -> Optional[int]:
        """First-fit reservation; returns the slot offset (its generation: :meth:`generation`)."""
        self._reap()
        n = -(-int(nbytes) // self.ALIGN) * self.ALIGN
        with self._lock:
            for r in self._free:
                if r[1] - r[0] >= n:
                    off = r[0]
                    r[0] += n
                    self._free = [x for x in self._free if x[1] > x[0]]
                    self._used[off] = n
                    self._reserved_at[off] = time.monotonic()
                    self._gen_of[off] = self._next_gen
                    self._next_gen += 1
                    return off
        return None

    def generation(self, offset: int) -> Optional[int]:
        with self._lock:
            return self._gen_of.get(int(offset))

    def release(self, offset: int, gen: Optional[int] = None) -> bool:
        """Free a slot. With ``gen``: only if it is still that reservation (a stale release is refused)."""
        with self._lock:
            offset = int(offset)
            if gen is not None and self._gen_of.get(offset) != int(gen):
                return False
            n = self._used.pop(offset, None)
            self._reserved_at.pop(offset, None)
            self._gen_of.pop(offset, None)
            if n is None:
                return False
            self._free.append([offset, offset + n])
            self._free.sort()
            merged: List[List[int]] = []
            for r in self._free:
                if merged and merged[-1][1] == r[0] and r[0] % self.seg_bytes:  # never across segments
                    merged[-1][1] = r[1]
                else:
                    merged.append(r)
            self._free = merged
            return True

    def claim(self, offset: int, shape: List[int], gen: Optional[int] = None) -> torch.Tensor:
        """A delivered packet as a bf16 view of its slot (the slot stays allocated until ``release_after``).
        ``gen``: the reservation's generation; an import for an expired reservation whose offset was
        reserved again is rejected (it would scatter the new owner's half-written bytes)."""
        offset = int(offset)
        n = int(np.prod(shape)) * 2
        with self._lock:
            if offset not in self._used or self._used[offset] < n:
                raise ValueError(f"kv_import of an unknown or too small landing-zone slot at {offset}")
            if gen is not None and self._gen_of.get(offset) != int(gen):
                raise ValueError(f"kv_import of a stale reservation at {offset} (generation {gen}, "
                                 f"slot now {self._gen_of.get(offset)})")
            self._reserved_at.pop(offset, None)  # imported: no longer expires
        seg, loc = divmod(offset, self.seg_bytes)
        return self.views[seg][loc: loc + n].view(torch.bfloat16).view(*shape)

    def release_after(self, offset: int, event=None) -> None:
        """Free the slot once ``event`` (recorded behind the consumer's scatter) has completed."""
        with self._lock:
            self._pending.append((int(offset), event))

    def take(self, offset: int, shape: List[int]) -> torch.Tensor:
        """Copy a delivered packet out of the zone and free its slot (tests / callers without a stream)."""
        kv = self.claim(offset, shape).clone()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.release_after(offset, ev)
        return kv

    def close(self) -> None:
        from src import _C

        self.views = []
        for p in self.ptrs:
            _C.car_release(p)
        self.ptrs = []


class IPCSender:
    """Prefill-worker side: maps a decode worker's :class:`IPCLandingZone` segments into this GPU's address
    space once. A slot reserved before the prompt ran is handed to the prefill engine as a tensor view
    (:meth:`dst`): the engine's export gathers the prompt's blocks straight into it. Otherwise a packed
    packet is copied in on a dedicated transfer stream (:meth:`write`), ordered after the engine's gather
    by its event; ``write_async`` / :meth:`wait_ready` await completion by polling (the asyncio thread
    never blocks on the GPU).

    ``dma = True`` copies with hipMemcpyAsync (copy engines) instead of the shader-store copy kernel: measured
    slower, and it slows a concurrent GEMM loop more (bench/micro_ipc_copy.py, profiles/micro_ipc_copy_r2.jsonl)."""

    def __init__(self, handles, seg_bytes: int, device):
        from src import _C

        if isinstance(handles, str):
            handles = [handles]
        self.device = torch.device(device)
        self.seg_bytes = int(seg_bytes)
        self.ptrs, self.views = [], []
        with torch.cuda.device(self.device):
            for h in handles:
                ptr = _C.car_open(bytes.fromhex(h))
                self.ptrs.append(ptr)
                self.views.append(_C.car_tensor(ptr, self.seg_bytes, self.device.index or 0))
            self.stream = torch.cuda.Stream(device=self.device)
        self.dma = False
        self.bytes_sent = 0

    def _loc(self, offset: int, nbytes: int):
        seg, loc = divmod(int(offset), self.seg_bytes)
        if seg >= len(self.ptrs) or loc + nbytes > self.seg_bytes:
            raise ValueError(f"slot at {offset} (+{nbytes} B) is outside the mapped landing zone")
        return seg, loc

    def dst(self, offset: int, shape: List[int]) -> torch.Tensor:
        """A bf16 view of the reserved slot (for the prefill engine's gather to write into)."""
        n = int(np.prod(shape)) * 2
        seg, loc = self._loc(offset, n)
        return self.views[seg][loc: loc + n].view(torch.bfloat16).view(*shape)

    def write(self, offset: int, kv: torch.Tensor, ready=None):
        from src import _C

        flat = kv.contiguous().view(torch.uint8).view(-1)
        seg, loc = self._loc(offset, flat.numel())
        s = self.stream
        with torch.cuda.device(self.device), torch.cuda.stream(s):
            if ready is not None:
                s.wait_event(ready)
            else:
                s.wait_stream(torch.cuda.current_stream(self.device))
            if self.dma:
                self.views[seg][loc: loc + flat.numel()].copy_(flat, non_blocking=True)
            else:  # shader stores into the mapped peer buffer
                _C.car_copy_to(self.ptrs[seg] + loc, flat)
            done = torch.cuda.Event()
            done.record(s)
        flat.record_stream(s)  # the staging tensor lives until the copy has read it
        self.bytes_sent += flat.numel()
        return done

    @staticmethod
    async def wait_ready(ev, poll_s: float = 2e-4) -> None:
        import asyncio

        while ev is not None and not ev.query():
            await asyncio.sleep(poll_s)

    async def write_async(self, offset: int, kv: torch.Tensor, ready=None, poll_s: float = 2e-4,
                          issued: Optional[Dict[str, Any]] = None) -> None:
        """Copy and wait for delivery without blocking the event loop. ``issued["event"]`` is set to the
        copy's completion event as soon as the copy is queued, so a caller that is cancelled while
        waiting knows the copy may still be writing into the slot."""
        done = self.write(offset, kv, ready)
        if issued is not None:
            issued["event"] = done
        await self.wait_ready(done, poll_s)

    def close(self) -> None:
        from src import _C

        self.views = []
        for p in self.ptrs:
            _C.car_close(p)
        self.ptrs = []


def packet_meta(p: KVPacket) -> Dict[str, Any]:
    """The packet without its KV payload (the IPC path writes the payload into the landing zone)."""
    return {"request_id": p.request_id, "prompt_ids": p.prompt_ids, "first_token": p.first_token,
            "shape": list(p.kv.shape), "block_size": p.block_size, "sampling": p.sampling, "ttft_ms": p.ttft_ms}


def packet_to_wire(p: KVPacket) -> Dict[str, Any]:
    kv = p.kv.detach().to("cpu").contiguous()
    raw = kv.view(torch.int16).numpy().tobytes()
    return {"request_id": p.request_id, "prompt_ids": p.prompt_ids, "first_token": p.first_token,
            "shape": list(kv.shape), "block_size": p.block_size, "sampling": p.sampling, "kv": raw,
            "ttft_ms": p.ttft_ms}


def packet_from_wire(d: Dict[str, Any], device="cpu") -> KVPacket:
    arr = np.frombuffer(d["kv"], dtype=np.int16).reshape(d["shape"])
    kv = torch.from_numpy(arr.copy()).view(torch.bfloat16).to(device)
    return KVPacket(d["request_id"], list(d["prompt_ids"]), int(d["first_token"]), kv, int(d["block_size"]),
                    dict(d.get("sampling") or {}), d.get("ttft_ms"))


class RCCLChannel:
    """Point-to-point KV shipping between two ranks of one process group
    (RCCL over xGMI on MI355X; gloo on CPU). A small int64 header carries the
    packet metadata, then the staging tensor follows."""

    HDR = 8

    def __init__(self, peer: int, device, group=None):
        self.peer = peer
        self.device = torch.device(device)
        self.group = group

    def send(self, p: KVPacket) -> None:
        n_ids = len(p.prompt_ids)
        hdr = torch.tensor([n_ids, p.first_token, p.block_size, *p.kv.shape, 0, 0][: self.HDR],
                           dtype=torch.int64, device=self.device)
        dist.send(hdr, self.peer, group=self.group)
        dist.send(torch.tensor(p.prompt_ids, dtype=torch.int64, device=self.device), self.peer, group=self.group)
        dist.send(p.kv.contiguous(), self.peer, group=self.group)

    def recv(self, request_id: str = "") -> KVPacket:
        hdr = torch.empty(self.HDR, dtype=torch.int64, device=self.device)
        dist.recv(hdr, self.peer, group=self.group)
        n_ids, first, bs, nb, planes, slab = (int(x) for x in hdr.tolist()[:6])
        ids = torch.empty(n_ids, dtype=torch.int64, device=self.device)
        dist.recv(ids, self.peer, group=self.group)
        kv = torch.empty(nb, planes, slab, dtype=torch.bfloat16, device=self.device)
        dist.recv(kv, self.peer, group=self.group)
        return KVPacket(request_id, ids.tolist(), first, kv, bs)
