"""
Configuration objects shared by every layer of the engine.

`ModelConfig` keeps the reference's six leading fields and their order
(`/root/reference/src/config.py:12-20`) so `ModelConfig("m", "/path", 8, 32)`
keeps working; everything after them is new and describes how a real model
session is placed on MI355X GPUs (architecture preset, dtype, tensor-parallel
degree, prefill/decode role, paged-KV geometry, HBM budget).

`EngineConfig` collects the continuous-batching scheduler knobs and
`DeploymentConfig` is the coordinator topology that `examples/demo_config.yaml`
(promised at `/root/reference/README.md:39`) is parsed into.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field, asdict
from typing import Any, Dict, List, Optional


@dataclass
class ModelConfig:
    """Configuration for a model served by a worker.

    The first six fields are the reference contract. `arch` selects the
    backend: ``"mock"`` (FakeModel echo, CPU), ``"llama"`` or ``"mixtral"``
    (GPU engine). `preset` names an architecture preset from
    :mod:`src.models.presets` (e.g. ``"llama3-8b"``); `model_path` may point at
    a safetensors directory, otherwise weights are random-initialised on device.
    """

    model_name: str
    model_path: str
    batch_size: int = 1
    max_batch_size: int = 32
    input_schema: Optional[Dict[str, Any]] = None
    output_schema: Optional[Dict[str, Any]] = None
    # --- MI355X engine extensions -------------------------------------------
    arch: str = "mock"
    preset: Optional[str] = None
    dtype: str = "bfloat16"
    tp_size: int = 1
    role: str = "both"                 # "prefill" | "decode" | "both"
    kv_block_size: int = 16
    max_model_len: int = 4096
    max_num_batched_tokens: int = 16384
    gpu_memory_fraction: float = 0.90
    num_kv_blocks: Optional[int] = None  # override the HBM-derived block count
    enable_prefix_caching: bool = True
    use_cuda_graph: bool = True        # hipGraph capture of decode steps
    max_latency_ms: float = 10.0
    seed: int = 0
    overrides: Dict[str, Any] = field(default_factory=dict)
    # text prompts / text outputs: 0 = tokenised and detokenised on the worker's event loop; N = in N separate
    # processes (src.preproc.PreprocPool). Token-id requests never touch the pool.
    preproc_processes: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ModelConfig":
        known = {f for f in cls.__dataclass_fields__}  # type: ignore[attr-defined]
        kwargs = {k: v for k, v in d.items() if k in known}
        extra = {k: v for k, v in d.items() if k not in known}
        cfg = cls(**kwargs)
        if extra:
            cfg.overrides.update(extra)
        return cfg


@dataclass
class EngineConfig:
    """Continuous-batching scheduler configuration (one engine per worker)."""

    max_num_seqs: int = 32
    max_num_batched_tokens: int = 16384
    max_latency_ms: float = 10.0       # admission wait bound (the reference Batcher knob)
    block_size: int = 16
    num_kv_blocks: Optional[int] = None
    gpu_memory_fraction: float = 0.90
    enable_prefix_caching: bool = True
    kv_block_ttl_s: Optional[float] = None  # TTL for cached (unreferenced) KV blocks
    use_cuda_graph: bool = True
    # padded decode batch sizes with a captured hipGraph (those above max_num_seqs are dropped)
    graph_batch_sizes: List[int] = field(default_factory=lambda: [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128])
    decode_partition_size: int = 256
    # decode steps replayed back to back on the GPU per host round trip when nothing is waiting
    # for admission (inputs advanced on the device; see src/engine/model_runner.py decode_multi)
    decode_window: int = 8
    # queue the next decode window behind the running one while the batch is unchanged, so the GPU
    # does not idle while the host applies a window's tokens (ModelRunner.decode_continue)
    async_decode: bool = True
    # KV-pool exhaustion during decode: "recompute" drops the victim's KV and re-prefills it later;
    # "swap" copies its blocks to pinned host memory and scatters them back on resume (no
    # recompute); "auto" swaps sequences with at least `swap_min_tokens` of context and recomputes
    # shorter ones (prefix-cached prompt blocks make those cheap). Swap space is host RAM.
    preemption_mode: str = "auto"
    swap_space_gib: float = 16.0
    swap_min_tokens: int = 256
    # prompts arriving while sequences decode (src/engine/scheduler.py): "auto" — prompt work that fits
    # in the decode step's spare rows (mixed_step_tokens - decode rows) rides along in ONE ragged batch
    # (a mixed step); more than that runs as a prefill step of at most prefill_tokens_while_decoding
    # tokens, and the next step decodes again (bounded stall). "always": every such step is mixed
    # (long prompts in mixed_step_tokens-row chunks); "off" (or False): prefill steps as before.
    # Measured on MI355X (profiles/poisson_r2.jsonl): 512-token prompts ride cheaper as whole prefill
    # steps than as 96-token chunks on the 128-row decode GEMM, short prompts ride along.
    mixed_batching: object = "auto"
    mixed_step_tokens: int = 64
    prefill_tokens_while_decoding: int = 4096
    # prefill batching under load: while sequences decode, newly arrived prompts that would need a
    # prefill step (not a mixed ride-along) are held until at least prefill_batch_tokens prompt tokens
    # wait or the oldest has waited prefill_batch_wait_ms — the reference Batcher's size-or-latency
    # flush (/root/reference/src/batcher.py:144-166) at the engine's admission point. Fewer, larger
    # prefill steps cost less per token (bench/micro_prefill_step.py: 20 us/token at 512 tokens, 12.9 at
    # 2,048), so decode is interrupted less; TTFT pays up to the wait. 0 disables.
    prefill_batch_tokens: int = 0
    prefill_batch_wait_ms: float = 60.0
    # disaggregated prefill: export each finishing prompt's KV per group of kv_export_group layers while the rest
    # of the forward runs (False: one gather after the step). Overlapped 48.95 vs 47.31 req/s
    # (profiles/disagg_r4_overlap_vs_not.jsonl)
    kv_export_overlap: bool = True
    kv_export_group: int = 4
    # disaggregated decode: single-step windows while imported prompts keep arriving (the last one less than
    # this long ago), so each joins at the next step instead of the next window (50.02 -> 50.65 req/s,
    # profiles/disagg_r4_import_settle_ab.jsonl). 0: off
    import_settle_ms: float = 3.0
    # open-loop arrivals: with two or more prompts arrived during decode within this lookback, no continuation
    # window is queued behind the running one (Poisson 40 req/s TTFT p50 38.6 -> 29.8 ms at equal e2e,
    # profiles/poisson_r4_arrival_ab.jsonl). 0: off
    arrival_window_ms: float = 250.0
    # prefill GEMMs: the measured solution table for the serving shapes (src/ops/gemm_table.py), read-only
    tuned_gemm_table: bool = True
    # decode-GEMM weight layout: "tiled" keeps tile-order copies of the dense projections beside prefill's
    # row-major weights (fastest decode; +13 GiB at Llama-3-8B / 32 rows), "single" runs the decode GEMMs on the
    # row-major weights (one copy: the bench 4 % slower, profiles/r5_decode_weight_layout_ab.txt, and that HBM goes
    # to the KV pool), "auto" = "single" when the KV pool is the constraint (kv_capacity_priority, or an explicit
    # num_kv_blocks that does not fit beside the copies), else "tiled". The choice is logged and in get_stats().
    decode_weight_layout: str = "auto"
    # the workload is bound by KV capacity (prefix-cache reuse under eviction: BASELINE config 5): every GiB of
    # HBM goes to the pool
    kv_capacity_priority: bool = False


@dataclass
class WorkerSpec:
    worker_id: str
    address: str
    shard_id: int = 0
    gpu: Optional[int] = None
    role: str = "both"


@dataclass
class DeploymentConfig:
    """Coordinator topology (models, shards, workers, strategies)."""

    listen_host: str = "127.0.0.1"
    listen_port: int = 9000
    strategy: str = "round_robin"
    batch_max_size: int = 32
    batch_max_latency_ms: float = 10.0
    # flush a partial batch once arrivals pause this long (closed-loop clients all waiting on it); 0: off
    batch_idle_flush_ms: float = 1.0
    cache_size: int = 10000
    cache_policy: str = "lru"
    cache_ttl_s: Optional[float] = None
    max_retries: int = 2
    request_timeout_s: float = 600.0
    health_check_interval: float = 5.0
    models: List[ModelConfig] = field(default_factory=list)
    workers: List[WorkerSpec] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "DeploymentConfig":
        d = dict(d)
        models = [ModelConfig.from_dict(m) for m in d.pop("models", [])]
        workers = [WorkerSpec(**w) for w in d.pop("workers", [])]
        known = {f for f in cls.__dataclass_fields__}  # type: ignore[attr-defined]
        cfg = cls(**{k: v for k, v in d.items() if k in known})
        cfg.models, cfg.workers = models, workers
        return cfg

    @classmethod
    def from_yaml(cls, path: str) -> "DeploymentConfig":
        import yaml

        with open(path) as f:
            data = yaml.safe_load(f) or {}
        return cls.from_dict(data)


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")
