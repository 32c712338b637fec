"""ModelRegistry: the behaviours `/root/reference/tests/test_registry.py`
checks (register/overwrite, add_shard + worker index, deterministic key→shard,
dict round-trip, versions, per-worker tracking) plus rendezvous remapping."""

import pytest

from src.model_registry import ModelRegistry, ModelStatus

MODEL = dict(model_name="m", version="1.0", model_path="/p", input_schema={"input": "float32"},
             output_schema={"output": "float32"}, batch_size=1, max_batch_size=32, quantized=False,
             metadata={"description": "t"})


@pytest.fixture
def reg():
    return ModelRegistry()


def test_register_and_overwrite(reg):
    reg.register_model(**MODEL)
    mv = reg.get_model_version("m", "1.0")
    assert mv.model_path == "/p" and reg.list_models() == ["m"]
    reg.register_model(**dict(MODEL, model_path="/q"))
    assert reg.get_model_version("m", "1.0").model_path == "/q"


def test_add_shard_indexes_worker(reg):
    reg.register_model(**MODEL)
    s = reg.add_shard("m", "1.0", shard_id=0, worker_id="w1", metadata={"gpu": "MI355X"})
    assert reg.get_model_version("m", "1.0").shards == [s]
    assert ("m", "1.0") in reg.get_worker_models("w1")
    assert reg.add_shard("m", "1.0", 0, "w9") is s          # idempotent on shard_id
    with pytest.raises(ValueError):
        reg.add_shard("nope", "1.0", 0, "w1")


@pytest.mark.parametrize("hashing", ["rendezvous", "modulo"])
def test_key_affinity(hashing):
    reg = ModelRegistry(hashing=hashing)
    reg.register_model(**MODEL)
    for i in range(3):
        reg.add_shard("m", "1.0", i, f"w{i}")
    a = reg.get_shard_for_key("m", "1.0", "user-1")
    assert a.shard_id == reg.get_shard_for_key("m", "1.0", "user-1").shard_id
    assert a.shard_id in (0, 1, 2)
    seen = {reg.get_shard_for_key("m", "1.0", f"k{i}").shard_id for i in range(200)}
    assert seen == {0, 1, 2}
    assert reg.get_shard_for_key("unknown", "1.0", "k") is None


def test_rendezvous_minimal_remap():
    reg = ModelRegistry()
    reg.register_model(**MODEL)
    for i in range(4):
        reg.add_shard("m", "1.0", i, f"w{i}")
    keys = [f"key{i}" for i in range(2000)]
    before = {k: reg.get_shard_for_key("m", "1.0", k).shard_id for k in keys}
    reg.add_shard("m", "1.0", 4, "w4")
    after = {k: reg.get_shard_for_key("m", "1.0", k).shard_id for k in keys}
    moved = [k for k in keys if before[k] != after[k]]
    assert all(after[k] == 4 for k in moved)          # only keys that now belong to the new shard move
    assert 0.1 < len(moved) / len(keys) < 0.3


def test_roundtrip(reg):
    reg.register_model(**MODEL)
    reg.add_shard("m", "1.0", 0, "w1", metadata={"tp_size": 8})
    reg.set_shard_status("m", "1.0", 0, ModelStatus.UPDATING, load=0.5)
    new = ModelRegistry.from_dict(reg.to_dict())
    a, b = reg.get_model_version("m", "1.0"), new.get_model_version("m", "1.0")
    assert a.to_dict() == b.to_dict()
    assert new.get_worker_models("w1") == [("m", "1.0")]
    assert new.get_model_hash("m", "1.0") == reg.get_model_hash("m", "1.0")


def test_versions(reg):
    for v in ("1.0", "1.1", "2.0"):
        reg.register_model(**dict(MODEL, version=v, model_path=f"/p/{v}"))
    assert reg.list_versions("m") == ["1.0", "1.1", "2.0"]
    assert reg.latest_version("m") == "2.0"
    for v in ("1.0", "1.1", "2.0"):
        assert reg.get_model_version("m", v).model_path == f"/p/{v}"


def test_worker_tracking(reg):
    for i in range(3):
        reg.register_model(**dict(MODEL, model_name=f"m{i}"))
        reg.add_shard(f"m{i}", "1.0", 0, "w0")
    reg.add_shard("m0", "1.0", 1, "w1")
    assert len(reg.get_worker_models("w0")) == 3
    assert reg.get_worker_models("w1") == [("m0", "1.0")]
    assert reg.get_worker_models("ghost") == []
    assert reg.remove_shard("m0", "1.0", 1) and reg.get_worker_models("w1") == []


def test_save_load(tmp_path, reg):
    reg.register_model(**MODEL)
    reg.add_shard("m", "1.0", 0, "w")
    p = str(tmp_path / "reg.json")
    reg.save(p)
    assert ModelRegistry.load(p).to_dict() == reg.to_dict()
