"""KVCache contract: the API `/root/reference/tests/test_kvstore.py` encodes
(close, item access, context manager, CacheEntry defaults, LRU, TTL) plus the
Appendix-B fixes (LRU with batch inserts, unknown policy rejected, LFU, FIFO,
persistence, thread safety)."""

import threading
import time

import pytest

from src.kvstore import CacheEntry, KVCache, KVStore, create_kv_store


@pytest.fixture
def kv():
    store = create_kv_store(max_size=3)
    yield store
    store.close()


def test_set_get_update_delete(kv):
    kv.set("a", 1)
    assert kv.get("a") == 1
    kv.set("a", 2)
    assert kv.get("a") == 2
    assert kv.get("zz") is None and kv.get("zz", "dflt") == "dflt"
    assert kv.delete("a") is True and kv.delete("a") is False
    kv["b"] = "B"
    assert "b" in kv and "nope" not in kv
    assert kv["b"] == "B"
    with pytest.raises(KeyError):
        kv["nope"]


def test_ttl_expiry(kv):
    kv.set("t", "v", ttl=0.05)
    assert kv.get("t") == "v"
    time.sleep(0.1)
    assert kv.get("t") is None
    assert "t" not in kv
    kv.set("p", "v", ttl=None)
    assert kv.get("p") == "v"


def test_default_ttl():
    s = KVCache(max_size=10, default_ttl=0.05)
    s.set("x", 1)
    time.sleep(0.1)
    assert len(s) == 0


def test_lru_eviction_order(kv):
    for k in ("k1", "k2", "k3"):
        kv.set(k, k.upper())
    kv.get("k1")                 # k1 becomes most recently used
    kv.set("k4", "K4")           # evicts k2
    assert kv.get("k2") is None
    assert [kv.get(k) for k in ("k1", "k3", "k4")] == ["K1", "K3", "K4"]
    assert len(kv) == 3
    assert kv.get_stats()["evictions"] == 1


def test_lru_with_batch_inserts_never_crashes():
    s = KVCache(max_size=2)
    s.batch_set({"a": 1, "b": 2})
    s.set("c", 3, batch=True)    # reference raised StopIteration here
    assert len(s) == 2 and s.get("c") == 3


def test_lfu_and_fifo():
    lfu = KVCache(max_size=2, eviction_policy="lfu")
    lfu.set("a", 1)
    lfu.set("b", 2)
    lfu.get("a"); lfu.get("a")
    lfu.set("c", 3)
    assert "b" not in lfu and "a" in lfu
    fifo = KVCache(max_size=2, eviction_policy="fifo")
    fifo.set("a", 1); fifo.set("b", 2); fifo.get("a"); fifo.set("c", 3)
    assert "a" not in fifo and "b" in fifo


def test_unknown_policy_rejected():
    with pytest.raises(ValueError):
        KVCache(eviction_policy="mru")


def test_context_manager_clears():
    with create_kv_store() as s:
        s["k"] = "v"
        assert s["k"] == "v"
    assert len(s) == 0 and s.get("k") is None


def test_values_stored_by_reference(kv):
    for i, v in enumerate(["s", 1, 2.5, True, None, {"k": 1}, [1, 2], (3, 4), {"x", "y"}]):
        kv.set(f"k{i}", v)
        assert kv.get(f"k{i}") == v


def test_cache_entry_defaults():
    now = time.time()
    e = CacheEntry(value="v", created_at=now, ttl=5)
    assert e.value == "v" and e.created_at == now and e.ttl == 5 and e.access_count == 0
    assert CacheEntry(value="v", created_at=now).ttl is None


def test_factory_defaults():
    s = create_kv_store()
    assert isinstance(s, KVStore) and s.max_size == 1000
    s.close()
    assert create_kv_store(max_size=7).max_size == 7


def test_stats_hit_rate(kv):
    kv.set("a", 1)
    kv.get("a"); kv.get("b")
    st = kv.get_stats()
    assert st["hits"] == 1 and st["misses"] == 1 and st["hit_rate"] == 0.5
    assert st["eviction_policy"] == "lru" and st["max_size"] == 3


def test_persistence_roundtrip(tmp_path):
    p = str(tmp_path / "kv.snap")
    s = KVCache(max_size=10, persist_path=p)
    s.set("a", {"v": 1}); s.set("b", [1, 2])
    s.close()
    s2 = KVCache(max_size=10, persist_path=p)
    assert s2.get("a") == {"v": 1} and s2.get("b") == [1, 2]


def test_persistence_is_json_not_pickle(tmp_path):
    """The snapshot is plain JSON (loading never executes file content); tuple keys survive,
    entries that are not JSON values are skipped rather than pickled."""
    import json

    p = str(tmp_path / "kv.snap")
    s = KVCache(max_size=10, persist_path=p)
    s.set(("llama", "1", 7), "x")
    s.set("obj", object())
    s.close()
    data = json.load(open(p))
    assert data["version"] == 2 and len(data["entries"]) == 1
    s2 = KVCache(max_size=10, persist_path=p)
    assert s2.get(("llama", "1", 7)) == "x" and s2.get("obj") is None


def test_thread_safety():
    s = KVCache(max_size=64)
    errs = []

    def work(t):
        try:
            for i in range(2000):
                s.set(f"{t}-{i % 100}", i)
                s.get(f"{(t + 1) % 4}-{i % 100}")
                if i % 7 == 0:
                    s.delete(f"{t}-{i % 50}")
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs and len(s) <= 64


def test_legacy_or_corrupt_snapshot_starts_empty(tmp_path):
    """A version-1 pickle snapshot (older build), a truncated file or foreign JSON must not stop the
    store (and so the coordinator) from starting; it is never unpickled."""
    import pickle

    cases = {
        "legacy.pkl": pickle.dumps({"version": 1, "entries": {"a": 1}}),
        "truncated.json": b'{"version": 2, "policy": "lru", "entries": [["a", 1',
        "foreign.json": b'["not", "a", "snapshot"]',
        "v3.json": b'{"version": 3, "entries": []}',
    }
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        store = KVCache(max_size=4, persist_path=str(p))
        assert len(store) == 0, name
        store.set("k", "v")
        store.close()  # the next save overwrites the bad file with a valid snapshot
        again = KVCache(max_size=4, persist_path=str(p))
        assert again.get("k") == "v", name
        again.close()
