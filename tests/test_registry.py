"""unittest suite for the model registry, runnable as the reference documents it
(``python -m unittest tests/test_registry.py -v``, tests/README.md) or under pytest.

Same behaviours as `/root/reference/tests/test_registry.py` (6 tests: register/overwrite,
shards + per-worker index, stable key -> shard, dict round trip, versions, worker
tracking); placement here is rendezvous hashing instead of md5 % N, so the key-stability
test also checks that adding a shard only moves keys to the new shard.
tests/test_model_registry.py has the pytest cases.
"""

import unittest

from src.model_registry import ModelRegistry

MODEL = {"model_name": "test_model", "version": "1.0", "model_path": "/models/test",
         "input_schema": {"input": "float32"}, "output_schema": {"output": "float32"},
         "batch_size": 1, "max_batch_size": 32, "quantized": False, "metadata": {"description": "t"}}


class TestModelRegistry(unittest.TestCase):
    def setUp(self):
        self.reg = ModelRegistry()

    def test_register_model(self):
        self.reg.register_model(**MODEL)
        mv = self.reg.get_model_version("test_model", "1.0")
        self.assertIsNotNone(mv)
        self.assertEqual((mv.version, mv.model_path), ("1.0", "/models/test"))
        self.assertEqual(len(self.reg.list_models()), 1)
        self.reg.register_model(**dict(MODEL, model_path="/models/v2"))   # same version: overwrite
        self.assertEqual(self.reg.get_model_version("test_model", "1.0").model_path, "/models/v2")

    def test_add_shard(self):
        self.reg.register_model(**MODEL)
        self.reg.add_shard(model_name="test_model", version="1.0", shard_id=0, worker_id="gpu-0",
                           metadata={"gpu": "MI355X"})
        shards = self.reg.get_model_version("test_model", "1.0").shards
        self.assertEqual([(s.shard_id, s.worker_id) for s in shards], [(0, "gpu-0")])
        self.assertIn(("test_model", "1.0"), self.reg.get_worker_models("gpu-0"))

    def test_get_shard_for_key(self):
        self.reg.register_model(**MODEL)
        for i in range(3):
            self.reg.add_shard(model_name="test_model", version="1.0", shard_id=i, worker_id=f"gpu-{i}")
        keys = [f"user-{i}" for i in range(200)]
        before = {k: self.reg.get_shard_for_key("test_model", "1.0", k).shard_id for k in keys}
        again = {k: self.reg.get_shard_for_key("test_model", "1.0", k).shard_id for k in keys}
        self.assertEqual(before, again)
        self.assertTrue(set(before.values()) <= {0, 1, 2})
        self.reg.add_shard(model_name="test_model", version="1.0", shard_id=3, worker_id="gpu-3")
        after = {k: self.reg.get_shard_for_key("test_model", "1.0", k).shard_id for k in keys}
        moved = [k for k in keys if after[k] != before[k]]
        self.assertTrue(all(after[k] == 3 for k in moved))

    def test_serialization(self):
        self.reg.register_model(**MODEL)
        self.reg.add_shard(model_name="test_model", version="1.0", shard_id=0, worker_id="gpu-0")
        copy = ModelRegistry.from_dict(self.reg.to_dict())
        self.assertEqual(set(copy.list_models()), set(self.reg.list_models()))
        a, b = self.reg.get_model_version("test_model", "1.0"), copy.get_model_version("test_model", "1.0")
        self.assertEqual((a.version, a.model_path, len(a.shards)), (b.version, b.model_path, len(b.shards)))
        self.assertEqual((a.shards[0].shard_id, a.shards[0].worker_id), (b.shards[0].shard_id, b.shards[0].worker_id))

    def test_model_versions(self):
        for v in ("1.0", "1.1", "2.0"):
            self.reg.register_model(**dict(MODEL, version=v, model_path=f"/models/{v}"))
        self.assertEqual(sorted(self.reg.list_versions("test_model")), ["1.0", "1.1", "2.0"])
        for v in ("1.0", "1.1", "2.0"):
            self.assertEqual(self.reg.get_model_version("test_model", v).model_path, f"/models/{v}")

    def test_worker_models(self):
        for i in range(3):
            self.reg.register_model(**dict(MODEL, model_name=f"m{i}"))
            self.reg.add_shard(model_name=f"m{i}", version="1.0", shard_id=0, worker_id="gpu-0")
        self.reg.add_shard(model_name="m0", version="1.0", shard_id=1, worker_id="gpu-1")
        self.assertEqual(len(self.reg.get_worker_models("gpu-0")), 3)
        self.assertEqual(set(self.reg.get_worker_models("gpu-1")), {("m0", "1.0")})
        self.assertEqual(len(self.reg.get_worker_models("nobody")), 0)


if __name__ == "__main__":
    unittest.main()
