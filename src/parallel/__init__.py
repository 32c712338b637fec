"""Distribution: tensor parallelism over RCCL/xGMI (:mod:`.tp`) and KV-block
transfer for disaggregated prefill/decode (:mod:`.kv_transfer`)."""

from .tp import TPContext, get_tp, init_tp  # noqa: F401
