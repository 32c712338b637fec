"""IPC landing-zone slot bookkeeping (host side, no device buffer): reservation generations make a
late kv_import / kv_release of an expired reservation harmless once its offset is reserved again
(ADVICE r2)."""

import time

import pytest
import torch

from src.parallel.kv_transfer import IPCLandingZone


def zone(cap=1 << 20, ttl=120.0, seg=None):
    z = object.__new__(IPCLandingZone)
    z.capacity = cap
    z.seg_bytes = seg or cap
    z.views = [torch.zeros(z.seg_bytes, dtype=torch.uint8) for _ in range(cap // z.seg_bytes)]
    z._init_book(ttl)
    return z


def test_generations_reject_stale_import_and_release():
    z = zone(ttl=0.05)
    a = z.reserve(1000)
    ga = z.generation(a)
    time.sleep(0.08)                 # reservation a expires (the sender stalled) ...
    b = z.reserve(1000)              # ... and first fit hands the same offset to another sender
    gb = z.generation(b)
    assert a == b and ga != gb and z.expired == 1
    with pytest.raises(ValueError, match="stale"):
        z.claim(a, [500], ga)        # the late kv_import of the first sender is rejected
    assert not z.release(a, ga)      # so is its late kv_release: b keeps its slot
    assert z.generation(b) == gb
    kv = z.claim(b, [500], gb)       # the current owner imports normally
    assert kv.dtype == torch.bfloat16 and kv.numel() == 500
    z.release_after(b, None)
    z._reap()
    assert not z._used and z._free == [[0, z.capacity]]


def test_release_without_generation_still_works():
    z = zone()
    o = z.reserve(4096)
    assert z.release(o) and not z.release(o)


def test_segments_slots_never_span_and_free_lists_stay_per_segment():
    """A multi-segment zone (several < 2 GiB IPC allocations): a slot lies inside one segment, claims map to
    that segment's buffer, and freeing never merges ranges across a segment boundary."""
    seg = 4 * IPCLandingZone.ALIGN
    z = zone(cap=3 * seg, seg=seg)
    a = z.reserve(3 * IPCLandingZone.ALIGN)          # segment 0, leaves one unit free there
    b = z.reserve(2 * IPCLandingZone.ALIGN)          # does not fit the rest of segment 0: segment 1
    c = z.reserve(IPCLandingZone.ALIGN)              # first fit: the tail of segment 0
    assert (a, b, c) == (0, seg, 3 * IPCLandingZone.ALIGN)
    assert z.reserve(5 * IPCLandingZone.ALIGN) is None   # larger than a segment: never
    kv = z.claim(b, [IPCLandingZone.ALIGN], z.generation(b))
    kv.fill_(1.0)
    assert z.views[1][: 2 * IPCLandingZone.ALIGN].view(torch.bfloat16).eq(1.0).all()
    assert z.views[0].eq(0).all()
    for o in (a, b, c):
        assert z.release(o)
    assert z._free == [[0, seg], [seg, 2 * seg], [2 * seg, 3 * seg]]
    # a whole bench wave of 32 x 64 MiB packets fits the default 4 x 1 GiB (one segment held only 16)
    # (bookkeeping only: no 4 GiB host buffer)
    z2 = object.__new__(IPCLandingZone)
    z2.capacity, z2.seg_bytes = 4 << 30, 1 << 30
    z2._init_book(120.0)
    offs = [z2.reserve(64 << 20) for _ in range(32)]
    assert None not in offs and len(set(offs)) == 32 and z2.reserve(2 << 30) is None


def test_export_slot_deadline_and_revocation():
    """a direct-export slot whose reservation may have expired on the decode side is never
    gathered into (the prompt queued / ran past the local deadline: staging tensor instead), and a revoked
    slot is never gathered into either; a slot revoked after its gather was queued reports the gather's
    event, so the sender releases it only behind that event."""
    from src.parallel.kv_transfer import ExportSlot

    calls = []

    def gather(dst):
        calls.append(dst)
        return ("slot" if dst is not None else "staging"), ("ev" if dst is not None else None)

    res = {"offset": 0, "gen": 1, "dst": "DST"}
    s = ExportSlot(res, deadline=time.monotonic() + 60)
    assert s.gather(gather) == ("slot", "ev") and s.state == "taken"
    assert s.revoke() == ("taken", "ev")
    s = ExportSlot(res, deadline=time.monotonic() - 1)       # past its deadline
    assert s.gather(gather) == ("staging", None) and s.state == "expired"
    assert s.revoke() == ("expired", None)
    s = ExportSlot(res, deadline=time.monotonic() + 60)
    assert s.revoke() == ("open", None) and s.state == "revoked"   # released at once by the sender
    assert s.gather(gather) == ("staging", None)
    assert calls == ["DST", None, None]


def test_remote_link_reserve_export_never_waits_and_revoke_releases():
    """The direct path reserves with wait_s=0 (a full zone must not hold prompts out of prefill) and takes
    its deadline from the decode worker's TTL; revoking an un-gathered slot releases it at once."""
    import asyncio

    from src.engine.disagg import RemoteDecodeLink

    async def main():
        link = RemoteDecodeLink("127.0.0.1:1", "m")
        sent = []

        class Ch:
            def dst(self, off, shape):
                return ("view", off)

        class RPC:
            async def call(self, addr, msg, timeout):
                sent.append(msg)
                if msg["op"] == "kv_reserve":
                    return {"success": True, "offset": 4096, "gen": 7, "ttl_s": 30.0}
                return {"success": True}

        link._ipc, link.rpc = Ch(), RPC()
        t0 = time.monotonic()
        slot = await link.reserve_export(torch.device("cpu"), [2, 4, 8])
        assert sent[0]["wait_s"] == 0.0 and sent[0]["nbytes"] == 2 * 2 * 4 * 8
        assert t0 + 30.0 - link.DEADLINE_MARGIN_S <= slot.deadline <= time.monotonic() + 30.0
        link.revoke(slot)
        await asyncio.sleep(0.01)
        assert sent[-1] == {"op": "kv_release", "model": "m", "offset": 4096, "gen": 7} and not link._tasks
    asyncio.run(main())


def test_remote_link_send_reserved_polls_then_imports():
    """A packet gathered straight into a reserved slot: the sender polls the gather's event (never blocks the
    event loop), then hands the slot over with ONE kv_import carrying only metadata (no event handle: the
    IPC-event hand-off measured slower and was removed in round 5)."""
    import asyncio

    from src.engine.disagg import RemoteDecodeLink
    from src.parallel.kv_transfer import KVPacket

    class Ev:
        def query(self):
            return True

    async def main():
        link = RemoteDecodeLink("127.0.0.1:1", "m")
        sent, polled = [], []

        class IPC:
            async def wait_ready(self, ev):
                polled.append(ev)

        class RPC:
            async def call(self, addr, msg, timeout):
                sent.append(msg)
                return {"success": True, "outputs": {}}

        link._ipc = IPC()
        link.rpc = RPC()
        pk = KVPacket("r", [1, 2], 5, torch.zeros(1, 2, 4, dtype=torch.bfloat16), 16, ready=Ev())
        rep = await link.send_reserved(pk, {"offset": 0, "gen": 3})
        assert rep["success"] and polled == [pk.ready] and len(sent) == 1
        assert sent[0]["op"] == "kv_import" and sent[0]["packet"]["ipc"] == {"offset": 0, "gen": 3}
        assert link.direct_packets == 1 and link.kv_path == "direct"
    asyncio.run(main())
