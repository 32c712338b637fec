"""Tensor parallelism on CPU (gloo, 2 ranks): the TP=2 engine (column/row
parallel linears, all-reduce, vocab-parallel LM head, rank-0-driven step
broadcast) must generate exactly what the TP=1 model with the same full
weights generates."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from src.config import EngineConfig
from src.engine import LLMEngine
from src.parallel.tp import TPContext
from src.parallel.tp_runner import build_tp_engine
from src.preproc import SamplingParams

PROMPTS = [[5, 9, 33, 12, 7] * 5, [100, 200, 300], list(range(3, 70))]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    return EngineConfig(max_num_seqs=4, max_num_batched_tokens=48, num_kv_blocks=64, max_latency_ms=0.0)


def _worker(rank, world, port, preset, q, moe_parallel="tp", sp=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext(rank=rank, world_size=world)
    try:
        obj = build_tp_engine(preset, tp, "cpu", cfg=_cfg(), max_model_len=256, capture=False,
                              dtype=torch.float32, full_init=True, seed=3, moe_parallel=moe_parallel,
                              sequence_parallel=sp)
        if rank == 0:
            obj.eos_token_id = None
            obj.runner.HEARTBEAT_S = 0.0  # idle heartbeats must be absorbed by the followers
            for _ in range(3):
                obj.runner.idle_tick()
            outs = obj.generate(PROMPTS, SamplingParams(max_tokens=6))
            obj.runner.stop_followers()
            q.put(outs)
        else:
            obj.follower_loop()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("preset,moe_parallel,sp", [("llama-tiny", "tp", False), ("mixtral-tiny", "tp", False),
                                                    ("mixtral-tiny", "ep", False), ("llama-tiny", "tp", True),
                                                    ("mixtral-tiny", "ep", True)])
def test_tp2_matches_tp1(preset, moe_parallel, sp):
    """TP=2; for Mixtral also expert parallelism (each rank owns half the experts, whole); with
    sequence parallelism the prefill's residual stream and norms are token-sharded (odd token
    counts exercise the padding)."""
    # TP=1 with full_init draws from the same rank-independent stream
    from src.models.llama import CausalLM
    from src.models.presets import get_preset
    m = CausalLM(get_preset(preset), "cpu", dtype=torch.float32, seed=3, max_position=256, full_init=True)
    ref = LLMEngine(m, _cfg(), 256)
    ref.eos_token_id = None
    expect = ref.generate(PROMPTS, SamplingParams(max_tokens=6))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, preset, q, moe_parallel, sp)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got == expect


def test_fused_exchange_residency_rule_at_70b_tp8_shapes():
    """CustomAllReduce.fused_ok: on an 8-GPU node (one rank per GPU, 256 CUs) the 70B TP=8 decode
    shard's row-parallel projections (wr = 32 tiles: o and down 256 column tiles, grid 256) carry the exchange
    in their GEMM epilogue because the whole grid is resident; with 8 ranks sharing ONE GPU the same shapes
    fall back to the separate all-reduce launch (neither the grid nor the waiting tiles fit), while 16 tiles
    (the one-GPU GPU test's shape) may still fuse."""
    from src.parallel.custom_allreduce import CustomAllReduce

    node = object.__new__(CustomAllReduce)
    node.ranks_per_gpu, node.cus = 1, 256
    assert node.fused_ok(256, grid=256)            # 8192 / 32 tiles, split-K 1
    assert node.fused_ok(128, grid=256)            # wr = 64, split-K 2
    assert not node.fused_ok(256, grid=512)        # a grid twice the CUs with every tile waiting: never
    shared = object.__new__(CustomAllReduce)
    shared.ranks_per_gpu, shared.cus = 8, 256
    assert not shared.fused_ok(256, grid=256) and not shared.fused_ok(128, grid=256)
    assert shared.fused_ok(16, grid=32)
