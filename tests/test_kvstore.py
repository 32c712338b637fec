"""unittest suite for the response cache (src/kvstore.py), runnable as
``python -m unittest tests/test_kvstore.py -v`` (tests/README.md) or under pytest.

It pins the API that `/root/reference/tests/test_kvstore.py` encodes — item access,
``close()``, context manager clearing on exit, ``CacheEntry`` defaults, LRU order, lazy TTL,
arbitrary value types, ``create_kv_store`` defaults — which the reference implementation
itself lacks (0/10 of those pass there). More detailed pytest cases are in
tests/test_kvstore_contract.py.
"""

import time
import unittest

from src.kvstore import CacheEntry, KVStore, create_kv_store


class TestKVStore(unittest.TestCase):
    def setUp(self):
        self.kv = create_kv_store(max_size=3)

    def tearDown(self):
        self.kv.close()

    def test_basic_operations(self):
        self.kv.set("k", "v")
        self.assertEqual(self.kv.get("k"), "v")
        self.kv.set("k", "v2")
        self.assertEqual(self.kv.get("k"), "v2")
        self.assertIsNone(self.kv.get("missing"))
        self.assertEqual(self.kv.get("missing", 7), 7)
        self.assertTrue(self.kv.delete("k"))
        self.assertFalse(self.kv.delete("k"))
        self.kv["x"] = 1
        self.assertIn("x", self.kv)
        self.assertNotIn("y", self.kv)

    def test_ttl(self):
        self.kv.set("short", 1, ttl=0.05)
        self.kv.set("forever", 2, ttl=None)
        self.assertEqual(self.kv.get("short"), 1)
        time.sleep(0.1)
        self.assertIsNone(self.kv.get("short"))
        self.assertNotIn("short", self.kv)
        self.assertEqual(self.kv.get("forever"), 2)

    def test_lru_eviction(self):
        for k in ("a", "b", "c"):
            self.kv.set(k, k.upper())
        self.kv.get("a")          # a becomes most recently used; b is now the LRU entry
        self.kv.set("d", "D")
        self.assertIsNone(self.kv.get("b"))
        self.assertEqual([self.kv.get(k) for k in ("a", "c", "d")], ["A", "C", "D"])
        self.assertEqual(len(self.kv), 3)

    def test_in_memory_lifetime_and_clear(self):
        kv = KVStore(max_size=10)
        kv.set("a", 1)
        kv.set("b", 2)
        self.assertEqual(len(kv), 2)
        kv.clear()
        self.assertEqual(len(kv), 0)
        self.assertIsNone(kv.get("a"))

    def test_context_manager_clears_on_exit(self):
        with create_kv_store() as kv:
            kv["a"] = 1
            self.assertEqual(kv["a"], 1)
        self.assertEqual(len(kv), 0)
        self.assertIsNone(kv.get("a"))

    def test_value_types(self):
        values = ["s", 1, 2.5, False, None, {"d": 1}, [1, 2], (3, 4), {"x", "y"}]
        for i, v in enumerate(values):
            self.kv.set(f"k{i}", v)
            self.assertEqual(self.kv.get(f"k{i}"), v)
            if i % 3 == 2:  # stay under max_size=3 so nothing is evicted mid-check
                self.kv.clear()

    def test_error_handling(self):
        kv = KVStore()
        self.assertIsNone(kv.get("missing"))
        self.assertFalse(kv.delete("missing"))
        with self.assertRaises(KeyError):
            kv["missing"]
        with self.assertRaises(ValueError):
            KVStore(eviction_policy="random")   # the reference silently fell back to FIFO

    def test_cache_entry_defaults(self):
        now = time.time()
        e = CacheEntry(value="v", created_at=now, ttl=60)
        self.assertEqual((e.value, e.created_at, e.ttl), ("v", now, 60))
        self.assertIsNone(CacheEntry(value="v", created_at=now).ttl)


class TestCreateKVStore(unittest.TestCase):
    def test_defaults(self):
        kv = create_kv_store()
        self.assertIsInstance(kv, KVStore)
        self.assertEqual(kv.max_size, 1000)
        kv.close()
        kv = create_kv_store(max_size=500)
        self.assertEqual(kv.max_size, 500)
        kv.close()


if __name__ == "__main__":
    unittest.main()
