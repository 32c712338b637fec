"""
Model registry: versions, shards and their placement.

API and JSON form follow `/root/reference/src/model_registry.py:20-249`
(``register_model``/``add_shard``/``get_shard_for_key``/``to_dict``/``from_dict`` …).

Differences:

* ``get_shard_for_key`` uses **rendezvous (highest-random-weight) hashing** by
  default, so adding or removing a shard only remaps the keys that belonged to
  it (the reference's "consistent hashing" was ``md5(key) % N`` over list
  position, `model_registry.py:158-161`). ``hashing="modulo"`` restores the
  reference behaviour.
* A shard group can hold **several workers**: on MI355X a "shard" is a
  placement unit — one data-parallel replica (a GPU), a tensor-parallel group
  (several GPUs acting as one), or a prefill/decode pair. ``ModelShard.metadata``
  carries ``{"tp_size", "gpus", "role"}``.
"""

from __future__ import annotations

import hashlib
import json
import logging
import struct
import threading
from dataclasses import dataclass, field
from enum import Enum, auto
from typing import Any, Dict, List, Optional, Set, Tuple

logger = logging.getLogger(__name__)


class ModelStatus(Enum):
    LOADING = auto()
    READY = auto()
    UPDATING = auto()
    FAILED = auto()
    UNLOADING = auto()


@dataclass
class ModelShard:
    shard_id: int
    worker_id: str
    status: ModelStatus = ModelStatus.READY
    load: float = 0.0
    metadata: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> Dict[str, Any]:
        return {
            "shard_id": self.shard_id,
            "worker_id": self.worker_id,
            "status": self.status.name,
            "load": self.load,
            "metadata": self.metadata,
        }


@dataclass
class ModelVersion:
    version: str
    model_path: str
    input_schema: Dict[str, Any]
    output_schema: Dict[str, Any]
    batch_size: int = 1
    max_batch_size: int = 32
    quantized: bool = False
    shards: List[ModelShard] = field(default_factory=list)
    metadata: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> Dict[str, Any]:
        return {
            "version": self.version,
            "model_path": self.model_path,
            "batch_size": self.batch_size,
            "max_batch_size": self.max_batch_size,
            "quantized": self.quantized,
            "shards": [s.to_dict() for s in self.shards],
            "input_schema": self.input_schema,
            "output_schema": self.output_schema,
            "metadata": self.metadata,
        }


def _key_digest(key: str) -> int:
    return int(hashlib.md5(key.encode()).hexdigest(), 16)


def rendezvous_score(key: str, shard_id: int) -> int:
    h = hashlib.blake2b(key.encode(), digest_size=8, person=b"die-hrw")
    h.update(struct.pack("<q", shard_id))
    return int.from_bytes(h.digest(), "little")


class ModelRegistry:
    """Stores model metadata keyed ``model_name -> version -> ModelVersion``."""

    def __init__(self, hashing: str = "rendezvous"):
        if hashing not in ("rendezvous", "modulo"):
            raise ValueError("hashing must be 'rendezvous' or 'modulo'")
        self.hashing = hashing
        self._models: Dict[str, Dict[str, ModelVersion]] = {}
        self._worker_models: Dict[str, Set[Tuple[str, str]]] = {}
        self._model_hashes: Dict[str, str] = {}
        self._lock = threading.RLock()

    # ---------------------------------------------------------------- models
    def register_model(
        self,
        model_name: str,
        version: str,
        model_path: str,
        input_schema: Optional[Dict[str, Any]] = None,
        output_schema: Optional[Dict[str, Any]] = None,
        batch_size: int = 1,
        max_batch_size: int = 32,
        quantized: bool = False,
        metadata: Optional[Dict[str, Any]] = None,
    ) -> ModelVersion:
        """Register (or overwrite) a model version. Re-registering drops its
        shards, as in the reference (`model_registry.py:86-114`)."""
        with self._lock:
            old = self._models.get(model_name, {}).get(version)
            if old is not None:
                for s in old.shards:
                    self._unindex(s.worker_id, model_name, version)
            mv = ModelVersion(
                version=version,
                model_path=model_path,
                input_schema=input_schema or {},
                output_schema=output_schema or {},
                batch_size=batch_size,
                max_batch_size=max_batch_size,
                quantized=quantized,
                metadata=metadata or {},
            )
            self._models.setdefault(model_name, {})[version] = mv
            self._update_model_hash(model_name, version)
            return mv

    def unregister_model(self, model_name: str, version: Optional[str] = None) -> bool:
        with self._lock:
            versions = self._models.get(model_name)
            if not versions:
                return False
            targets = [version] if version else list(versions)
            found = False
            for v in targets:
                mv = versions.pop(v, None)
                if mv is None:
                    continue
                found = True
                for s in mv.shards:
                    self._unindex(s.worker_id, model_name, v)
                self._model_hashes.pop(f"{model_name}:{v}", None)
            if not versions:
                self._models.pop(model_name, None)
            return found

    # ---------------------------------------------------------------- shards
    def add_shard(
        self,
        model_name: str,
        version: str,
        shard_id: int,
        worker_id: str,
        metadata: Optional[Dict[str, Any]] = None,
    ) -> ModelShard:
        with self._lock:
            mv = self.get_model_version(model_name, version)
            if mv is None:
                raise ValueError(f"Model {model_name} version {version} not found")
            existing = next((s for s in mv.shards if s.shard_id == shard_id), None)
            if existing is not None:
                return existing
            shard = ModelShard(shard_id=shard_id, worker_id=worker_id, metadata=metadata or {})
            mv.shards.append(shard)
            self._worker_models.setdefault(worker_id, set()).add((model_name, version))
            return shard

    def remove_shard(self, model_name: str, version: str, shard_id: int) -> bool:
        with self._lock:
            mv = self.get_model_version(model_name, version)
            if mv is None:
                return False
            for i, s in enumerate(mv.shards):
                if s.shard_id == shard_id:
                    mv.shards.pop(i)
                    if not any(o.worker_id == s.worker_id for o in mv.shards):
                        self._unindex(s.worker_id, model_name, version)
                    return True
            return False

    def set_shard_status(self, model_name: str, version: str, shard_id: int,
                         status: ModelStatus, load: Optional[float] = None) -> None:
        with self._lock:
            mv = self.get_model_version(model_name, version)
            if mv is None:
                return
            for s in mv.shards:
                if s.shard_id == shard_id:
                    s.status = status
                    if load is not None:
                        s.load = load

    def get_shard_for_key(self, model_name: str, version: str, key: str) -> Optional[ModelShard]:
        """Deterministic key → shard placement (session affinity)."""
        with self._lock:
            mv = self.get_model_version(model_name, version)
            if mv is None or not mv.shards:
                return None
            return self.pick_shard(mv.shards, key)

    def pick_shard(self, shards: List[ModelShard], key: str) -> ModelShard:
        if self.hashing == "modulo":
            return shards[_key_digest(key) % len(shards)]
        return max(shards, key=lambda s: rendezvous_score(key, s.shard_id))

    # --------------------------------------------------------------- queries
    def get_model_version(self, model_name: str, version: str) -> Optional[ModelVersion]:
        return self._models.get(model_name, {}).get(version)

    def latest_version(self, model_name: str) -> Optional[str]:
        versions = self.list_versions(model_name)
        return versions[-1] if versions else None

    def list_models(self) -> List[str]:
        return list(self._models.keys())

    def list_versions(self, model_name: str) -> List[str]:
        return list(self._models.get(model_name, {}).keys())

    def get_worker_models(self, worker_id: str) -> List[Tuple[str, str]]:
        return list(self._worker_models.get(worker_id, set()))

    def _unindex(self, worker_id: str, model_name: str, version: str) -> None:
        s = self._worker_models.get(worker_id)
        if s is not None:
            s.discard((model_name, version))
            if not s:
                del self._worker_models[worker_id]

    def _update_model_hash(self, model_name: str, version: str) -> None:
        d = self._models[model_name][version].to_dict()
        d["shards"] = []
        self._model_hashes[f"{model_name}:{version}"] = hashlib.md5(
            json.dumps(d, sort_keys=True, default=str).encode()).hexdigest()

    def get_model_hash(self, model_name: str, version: str) -> Optional[str]:
        return self._model_hashes.get(f"{model_name}:{version}")

    # --------------------------------------------------------- serialization
    def to_dict(self) -> Dict[str, Any]:
        with self._lock:
            return {
                "hashing": self.hashing,
                "models": {
                    name: {v: mv.to_dict() for v, mv in versions.items()}
                    for name, versions in self._models.items()
                },
            }

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "ModelRegistry":
        reg = cls(hashing=data.get("hashing", "rendezvous"))
        for name, versions in data.get("models", {}).items():
            for vstr, md in versions.items():
                shards = [
                    ModelShard(
                        shard_id=sd["shard_id"],
                        worker_id=sd["worker_id"],
                        status=ModelStatus[sd.get("status", "READY")],
                        load=sd.get("load", 0.0),
                        metadata=sd.get("metadata", {}),
                    )
                    for sd in md.get("shards", [])
                ]
                mv = ModelVersion(
                    version=md["version"],
                    model_path=md["model_path"],
                    input_schema=md.get("input_schema", {}),
                    output_schema=md.get("output_schema", {}),
                    batch_size=md.get("batch_size", 1),
                    max_batch_size=md.get("max_batch_size", 32),
                    quantized=md.get("quantized", False),
                    shards=shards,
                    metadata=md.get("metadata", {}),
                )
                reg._models.setdefault(name, {})[vstr] = mv
                reg._update_model_hash(name, vstr)
                for s in shards:
                    reg._worker_models.setdefault(s.worker_id, set()).add((name, vstr))
        return reg

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2, default=str)

    @classmethod
    def load(cls, path: str) -> "ModelRegistry":
        with open(path) as f:
            return cls.from_dict(json.load(f))
