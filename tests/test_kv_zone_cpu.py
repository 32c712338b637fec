"""IPC landing-zone slot bookkeeping (host side, no device buffer): reservation generations make a
late kv_import / kv_release of an expired reservation harmless once its offset is reserved again
(ADVICE r2)."""

import time

import pytest
import torch

from src.parallel.kv_transfer import IPCLandingZone


def zone(cap=1 << 20, ttl=120.0):
    z = object.__new__(IPCLandingZone)
    z.capacity = cap
    z.view = torch.zeros(cap, dtype=torch.uint8)
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
