"""
Key-value stores.

Two caches live here, one per level of the serving stack:

* :class:`KVCache` — the request/response cache the coordinator consults before
  dispatching (`/root/reference/src/kvstore.py:26-236`). Same public API and
  statistics as the reference, plus the contract its test-suite encodes
  (`/root/reference/tests/test_kvstore.py`: ``close()``, ``kv[k]`` with
  ``KeyError`` on a miss, ``kv[k] = v``, a context manager that clears on exit,
  ``CacheEntry`` constructible without ``last_accessed``) and the fixes listed
  in SURVEY Appendix B: a real lock, LRU that survives ``batch=True`` inserts,
  unknown policies rejected instead of silently acting as FIFO, and optional
  on-disk persistence (`README.md:14,89`).

* :class:`PagedKVCache` — the GPU KV-block cache: the "kvstore" of the MI355X
  engine. Blocks live in HBM (one pool tensor for all layers, see
  :class:`src.engine.model_runner.KVPool`); bookkeeping (free list, ref-counts,
  prefix-hash index and LRU/TTL eviction of unreferenced cached blocks) is the
  native C++ block manager (``csrc/runtime/block_manager.h``, bound in
  ``src/_runtime``). It exposes the
  same ``get/set/delete/get_stats`` verbs over block hashes so the coordinator
  and the engine speak one cache vocabulary.
"""

from __future__ import annotations

import json
import logging
import os
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Dict, Generic, Iterable, List, Optional, TypeVar

T = TypeVar("T")
logger = logging.getLogger(__name__)


def _freeze(x):
    """JSON arrays back to hashable keys (tuples, recursively)."""
    return tuple(_freeze(v) for v in x) if isinstance(x, list) else x

_POLICIES = ("lru", "lfu", "fifo")


@dataclass
class CacheEntry(Generic[T]):
    """A cached value plus bookkeeping (reference `kvstore.py:17-24`)."""

    value: T
    created_at: float
    last_accessed: float = field(default_factory=time.time)
    access_count: int = 0
    ttl: Optional[float] = None  # seconds

    def expired(self, now: Optional[float] = None) -> bool:
        if self.ttl is None:
            return False
        return ((now if now is not None else time.time()) - self.created_at) > self.ttl


class KVCache:
    """Thread-safe in-memory cache with LRU / LFU / FIFO eviction and TTLs.

    Eviction removes one victim when an insert would exceed ``max_size``
    (reference `kvstore.py:82-102`). TTL expiry is lazy (on access) as in the
    reference, plus :meth:`purge_expired` for an explicit sweep.
    """

    def __init__(
        self,
        max_size: int = 1000,
        eviction_policy: str = "lru",
        default_ttl: Optional[float] = None,
        persist_path: Optional[str] = None,
    ):
        policy = eviction_policy.lower()
        if policy not in _POLICIES:
            raise ValueError(f"unknown eviction policy {eviction_policy!r}; expected one of {_POLICIES}")
        if max_size < 1:
            raise ValueError("max_size must be >= 1")
        self.max_size = max_size
        self.eviction_policy = policy
        self.default_ttl = default_ttl
        self.persist_path = persist_path
        # Insertion-ordered for FIFO, access-ordered for LRU (move_to_end on touch).
        self.cache: "OrderedDict[Any, CacheEntry]" = OrderedDict()
        self._lock = threading.RLock()
        self._closed = False
        self.hits = 0
        self.misses = 0
        self.evictions = 0
        if persist_path and os.path.exists(persist_path):
            try:
                self.load(persist_path)
            except (OSError, UnicodeDecodeError, ValueError, TypeError, KeyError) as e:
                # a version-1 (pickle) snapshot of an older build, or a truncated / foreign file: start
                # empty rather than fail the coordinator at startup (never fall back to unpickling it)
                logger.warning("KVCache: ignoring unreadable snapshot %s (%s); starting empty", persist_path, e)
                self.cache.clear()

    # ------------------------------------------------------------------ core
    def _victim(self):
        if self.eviction_policy == "lfu":
            # Least access_count, ties broken by oldest access.
            return min(self.cache.items(), key=lambda kv: (kv[1].access_count, kv[1].last_accessed))[0]
        # LRU: front of access order; FIFO: front of insertion order.
        return next(iter(self.cache))

    def _evict_if_needed(self) -> None:
        while len(self.cache) >= self.max_size:
            # Prefer dropping an expired entry over a live one.
            now = time.time()
            expired = next((k for k, e in self.cache.items() if e.expired(now)), None)
            key = expired if expired is not None else self._victim()
            del self.cache[key]
            self.evictions += 1

    def set(self, key, value, ttl: Optional[float] = None, batch: bool = False) -> None:
        """Insert or replace ``key``. ``batch`` is accepted for API parity; the
        access order is always maintained so LRU never loses track of a key."""
        with self._lock:
            now = time.time()
            if key in self.cache:
                del self.cache[key]
            self._evict_if_needed()
            self.cache[key] = CacheEntry(
                value=value,
                created_at=now,
                last_accessed=now,
                ttl=ttl if ttl is not None else self.default_ttl,
            )

    def get(self, key, default: Any = None) -> Any:
        with self._lock:
            entry = self.cache.get(key)
            if entry is None:
                self.misses += 1
                return default
            if entry.expired():
                del self.cache[key]
                self.misses += 1
                return default
            entry.last_accessed = time.time()
            entry.access_count += 1
            if self.eviction_policy == "lru":
                self.cache.move_to_end(key)
            self.hits += 1
            return entry.value

    def exists(self, key) -> bool:
        return key in self

    def batch_get(self, keys: Iterable) -> Dict[Any, Any]:
        with self._lock:
            return {k: self.get(k) for k in keys}

    def batch_set(self, items: Dict[Any, Any], ttl: Optional[float] = None) -> None:
        with self._lock:
            for k, v in items.items():
                self.set(k, v, ttl=ttl, batch=True)

    def delete(self, key) -> bool:
        with self._lock:
            if key in self.cache:
                del self.cache[key]
                return True
            return False

    def clear(self) -> None:
        with self._lock:
            self.cache.clear()
            self.hits = self.misses = self.evictions = 0

    def purge_expired(self) -> int:
        with self._lock:
            now = time.time()
            dead = [k for k, e in self.cache.items() if e.expired(now)]
            for k in dead:
                del self.cache[k]
            return len(dead)

    def get_stats(self) -> Dict[str, Any]:
        with self._lock:
            total = self.hits + self.misses
            return {
                "hits": self.hits,
                "misses": self.misses,
                "hit_rate": self.hits / total if total else 0.0,
                "size": len(self.cache),
                "max_size": self.max_size,
                "evictions": self.evictions,
                "eviction_policy": self.eviction_policy,
            }

    # ------------------------------------------------------------ persistence
    def save(self, path: Optional[str] = None) -> str:
        """Snapshot live entries to ``path`` as JSON (keys and values must be JSON values; tuple
        keys come back as tuples). Entries that are not JSON-serialisable are skipped. JSON, not
        pickle: loading a snapshot never executes anything from the file."""
        path = path or self.persist_path
        if not path:
            raise ValueError("no persist path configured")
        with self._lock:
            now = time.time()
            snap = [(k, e.value, e.created_at, e.ttl) for k, e in self.cache.items() if not e.expired(now)]
        entries, skipped = [], 0
        for k, v, created, ttl in snap:
            try:
                entries.append(json.dumps([k, v, created, ttl]))
            except (TypeError, ValueError):
                skipped += 1
        if skipped:
            logger.warning("KVCache.save: %d entries are not JSON-serialisable and were not saved", skipped)
        tmp = f"{path}.tmp"
        with open(tmp, "w") as f:
            f.write('{"version": 2, "policy": %s, "entries": [%s]}' % (json.dumps(self.eviction_policy),
                                                                        ", ".join(entries)))
        os.replace(tmp, path)
        return path

    def load(self, path: Optional[str] = None) -> int:
        """Restore a JSON snapshot written by :meth:`save`."""
        path = path or self.persist_path
        with open(path, encoding="utf-8") as f:
            data = json.load(f)
        if not isinstance(data, dict) or data.get("version") != 2:
            raise ValueError(f"{path}: not a version-2 JSON KVCache snapshot")
        n = 0
        with self._lock:
            now = time.time()
            for key, value, created_at, ttl in data.get("entries", []):
                e = CacheEntry(value=value, created_at=created_at, last_accessed=now, ttl=ttl)
                if e.expired(now):
                    continue
                self._evict_if_needed()
                self.cache[_freeze(key)] = e
                n += 1
        return n

    def close(self) -> None:
        if self._closed:
            return
        if self.persist_path:
            try:
                self.save()
            except OSError:
                pass
        self._closed = True

    # -------------------------------------------------------------- dunders
    def __getitem__(self, key):
        sentinel = _MISSING
        v = self.get(key, sentinel)
        if v is sentinel:
            raise KeyError(key)
        return v

    def __setitem__(self, key, value) -> None:
        self.set(key, value)

    def __delitem__(self, key) -> None:
        if not self.delete(key):
            raise KeyError(key)

    def __contains__(self, key) -> bool:
        with self._lock:
            e = self.cache.get(key)
            if e is None:
                return False
            if e.expired():
                del self.cache[key]
                return False
            return True

    def __len__(self) -> int:
        with self._lock:
            self.purge_expired()
            return len(self.cache)

    def __enter__(self) -> "KVCache":
        return self

    def __exit__(self, *exc) -> None:
        self.clear()
        self.close()

    def __repr__(self) -> str:
        return f"KVCache(size={len(self.cache)}, max_size={self.max_size}, policy={self.eviction_policy})"


_MISSING = object()

# Reference aliases (`kvstore.py:238-240`).
KVStore = KVCache


def create_kv_store(max_size: int = 1000, eviction_policy: str = "lru", default_ttl: Optional[float] = None,
                    persist_path: Optional[str] = None) -> KVCache:
    return KVCache(max_size=max_size, eviction_policy=eviction_policy, default_ttl=default_ttl,
                   persist_path=persist_path)


class PagedKVCache:
    """GPU paged KV-block cache (HBM blocks + native block manager).

    This is a façade: ``allocate``/``free``/``match_prefix`` go straight to the
    C++ :class:`BlockManager`; ``get/set/delete`` operate on *prefix hashes*
    (hash of a full block of token ids chained with its parent's hash) so a
    cached prompt prefix can be looked up like any other cache key.
    The device tensors are owned by :class:`src.engine.model_runner.KVPool`.
    """

    def __init__(self, num_blocks: int, block_size: int, enable_prefix_caching: bool = True,
                 ttl_s: Optional[float] = None, pool=None):
        from src.engine.block_manager import BlockManager

        self.block_size = block_size
        self.num_blocks = num_blocks
        self.manager = BlockManager(num_blocks, block_size, enable_prefix_caching, ttl_s)
        self.pool = pool

    # cache vocabulary over prefix hashes
    def get(self, block_hash: int, default=None):
        b = self.manager.lookup(block_hash)
        return default if b < 0 else b

    def set(self, block_hash: int, block_id: int) -> None:
        self.manager.register(block_hash, block_id)

    def delete(self, block_hash: int) -> bool:
        return self.manager.forget(block_hash)

    def __contains__(self, block_hash: int) -> bool:
        return self.manager.lookup(block_hash) >= 0

    # allocator vocabulary
    def allocate(self, n: int) -> List[int]:
        return self.manager.allocate(n)

    def free(self, blocks: List[int]) -> None:
        self.manager.free(blocks)

    def get_stats(self) -> Dict[str, Any]:
        s = self.manager.stats()
        if self.pool is not None:
            s["hbm_bytes"] = self.pool.nbytes
        return s
