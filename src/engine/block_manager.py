"""
Per-sequence KV block accounting on top of the native C++ block manager
(``csrc/runtime/block_manager.h``): prompt allocation with automatic prefix
caching, one-slot growth during decode, release (to the free stack or the
evictable LRU of cached prefix blocks), and TTL sweeps.
"""

from __future__ import annotations

from typing import List, Optional

from src.engine.sequence import Sequence

try:
    from src import _runtime  # type: ignore
except Exception as e:  # pragma: no cover
    _runtime = None
    _RUNTIME_ERR = e


def _native():
    if _runtime is None:
        # The host runtime is plain C++ (g++); build it in place on first use.
        from src._build import build_runtime
        import importlib

        build_runtime()
        return importlib.import_module("src._runtime")
    return _runtime


def BlockManager(num_blocks: int, block_size: int, prefix_caching: bool = True, ttl_s: Optional[float] = None):
    return _native().BlockManager(num_blocks, block_size, prefix_caching, -1.0 if ttl_s is None else float(ttl_s))


def native_runtime():
    return _native()


class KVBlockManager:
    def __init__(self, num_blocks: int, block_size: int, enable_prefix_caching: bool = True,
                 ttl_s: Optional[float] = None, salt: int = 0):
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.prefix_caching = enable_prefix_caching
        self.salt = salt
        self.bm = BlockManager(num_blocks, block_size, enable_prefix_caching, ttl_s)
        self._hash = _native().BlockManager.hash_blocks

    # ----------------------------------------------------------- queries
    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    def num_available(self) -> int:
        return self.bm.num_available()

    def usage(self) -> float:
        return self.bm.num_used() / self.num_blocks

    # -------------------------------------------------------- allocation
    def _prompt_hashes(self, seq: Sequence) -> List[int]:
        if seq.block_hashes is None:
            seq.block_hashes = list(self._hash(seq.prompt_ids, self.block_size, 0, self.salt))
        return seq.block_hashes

    def can_allocate(self, seq: Sequence, reserve: int = 0) -> bool:
        return self.blocks_needed(len(seq)) + reserve <= self.bm.num_available()

    def allocate(self, seq: Sequence) -> None:
        """Give ``seq`` blocks for all of its current tokens, reusing cached
        prefix blocks. At least the last prompt token is always recomputed
        (its logits are needed), so at most ``(len-1)//bs`` blocks are matched."""
        assert not seq.block_table
        matched: List[int] = []
        if self.prefix_caching and not seq.imported_kv:
            hashes = self._prompt_hashes(seq)
            max_match = (seq.prompt_len - 1) // self.block_size
            matched = list(self.bm.match_prefix(hashes[:max_match]))
        need = self.blocks_needed(len(seq)) - len(matched)
        try:
            fresh = list(self.bm.allocate(need))
        except RuntimeError:
            if matched:
                self.bm.free(matched)
            raise
        seq.block_table = matched + fresh
        seq.num_computed = len(matched) * self.block_size
        seq.num_prefix_hit = seq.num_computed

    def allocate_fresh(self, seq: Sequence, n_blocks: int) -> List[int]:
        """A table of ``n_blocks`` new blocks (no prefix matching): swap-in target."""
        assert not seq.block_table
        seq.block_table = list(self.bm.allocate(n_blocks))
        return list(seq.block_table)

    def ensure_slots(self, seq: Sequence, n_tokens: int) -> bool:
        """Grow the table to hold ``n_tokens`` tokens. False if out of blocks."""
        need = self.blocks_needed(n_tokens) - len(seq.block_table)
        if need <= 0:
            return True
        if need > self.bm.num_available():
            return False
        seq.block_table.extend(self.bm.allocate(need))
        return True

    def register_prompt_blocks(self, seq: Sequence) -> None:
        """Publish the full blocks of a computed prompt to the prefix cache."""
        if not self.prefix_caching:
            return
        hashes = self._prompt_hashes(seq)
        n = min(len(hashes), seq.num_computed // self.block_size)
        for i in range(n):
            self.bm.register_block(hashes[i], seq.block_table[i])

    def free(self, seq: Sequence) -> None:
        if seq.block_table:
            self.bm.free(seq.block_table)
        seq.block_table = []

    def evict_expired(self) -> int:
        return self.bm.evict_expired()

    def stats(self) -> dict:
        s = dict(self.bm.stats())
        s["usage"] = self.usage()
        return s
