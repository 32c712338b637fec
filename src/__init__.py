"""
MI355X-native distributed inference engine.

Control plane (reference layout, `/root/reference/src/`): ``config``,
``kvstore``, ``model_registry``, ``router``, ``load_balancer``, ``batcher``,
``worker``, ``coordinator``, ``preproc``, ``postproc``, ``utils``,
``mock_models``. Data plane (new): ``engine`` (paged KV, continuous batching,
hipGraph decode), ``models`` (Llama-3, Mixtral), ``ops`` (hand-written
gfx950 HIP kernels), ``parallel`` (tensor parallel over RCCL/xGMI, KV-block
transfer).
"""

from .kvstore import KVStore, create_kv_store  # noqa: F401

__all__ = ["KVStore", "create_kv_store"]
__version__ = "0.1.0"
