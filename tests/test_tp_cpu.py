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
    """The exchange fused into the row-parallel decode GEMM (custom_allreduce.fused_exchange_ok, VERDICT r5 weak 5 /
    ADVICE r5): on an 8-GPU node (one rank per GPU, 256 CUs) the 70B TP=8 shard's o / down at 32 rows (wr = 32:
    256 column tiles, grid 256) do NOT fuse with the full LDS ring (one workgroup per CU: 256 > 256 - margin, and
    256 waiting tiles would hold every CU) — a single CU held by another stream could stall the grid — but do with
    the half-LDS ring (two per CU: 256 <= 512 - 16). wr = 64 tiles (128 waiters <= half the CUs) always may. With
    8 ranks sharing ONE GPU the same shapes fall back to the separate all-reduce launch; 16 tiles may still fuse."""
    from src.parallel.custom_allreduce import CustomAllReduce, fused_exchange_ok, residency_margin

    assert residency_margin(256) == 16
    node = object.__new__(CustomAllReduce)
    node.ranks_per_gpu, node.cus = 1, 256
    assert not node.fused_ok(256, grid=256, per_cu=1)   # 8192 / 32 tiles, full ring: zero slack -> separate
    assert node.fused_ok(256, grid=256, per_cu=2)       # the half-LDS ring: 256 <= 496
    assert not node.fused_ok(256, grid=256)             # occupancy unknown: only rule (b), which fails
    assert node.fused_ok(128, grid=256, per_cu=1)       # wr = 64, split-K 2: 128 waiters <= 128
    assert not node.fused_ok(256, grid=512, per_cu=2)   # 512 > 496 and 256 waiters
    assert node.fused_ok(256, grid=512, per_cu=3)
    assert not fused_exchange_ok(300, 300, 4, 1, 256)   # more tiles than flag slots
    shared = object.__new__(CustomAllReduce)
    shared.ranks_per_gpu, shared.cus = 8, 256
    assert not shared.fused_ok(256, grid=256, per_cu=2) and not shared.fused_ok(128, grid=256, per_cu=1)
    assert shared.fused_ok(16, grid=32, per_cu=1)
    # ranks sharing a GPU: small-ring waiters on every CU would starve another rank's full-LDS kernel, so the
    # occupancy counts as one per CU there, without margin (the rule the one-GPU suite validated in round 5)
    assert shared.fused_ok(32, grid=32, per_cu=2) and not shared.fused_ok(33, grid=33, per_cu=2)
    four = object.__new__(CustomAllReduce)
    four.ranks_per_gpu, four.cus = 4, 256
    assert four.fused_ok(32, grid=32, per_cu=2) and four.fused_ok(32, grid=32, per_cu=1)


def test_tp_plan_takes_a_residency_safe_tile(monkeypatch):
    """decode_plan under TP: the measured wr = 32 tile with the half-LDS ring when the full ring fails the rule, a
    wider tile when no half ring exists, the separate launch when nothing passes (occupancy stubbed: no GPU here)."""
    from src import ops
    from src.models.llama import CausalLM
    from src.models.presets import get_preset
    from src.parallel.tp import TPContext

    class NodeTP(TPContext):  # one rank per GPU on a 256-CU node, the IPC path assumed up
        def fused_row_parallel(self, n_tiles, grid=0, per_cu=0):
            from src.parallel.custom_allreduce import fused_exchange_ok
            return fused_exchange_ok(n_tiles, grid, per_cu, 1, 256)

    m = object.__new__(CausalLM)
    m.arch = get_preset("llama3-70b")
    m.tp = NodeTP(rank=0, world_size=8)
    m.hq, m.hkv, m.head_dim, m.inter = 8, 1, 128, 28672 // 8
    m.layers = [type("L", (), {"qkv": torch.empty(1280, 8192, device="meta")})()]
    occ = {False: 1, True: 2}
    monkeypatch.setattr(ops, "gd_occupancy", lambda mode, wr, kc, sk, rows, half=False: occ[half])
    p = m.decode_plan(32)
    assert p["tp_fused"] and p["o"][0] == 32 and p["o_half"] and p["down_half"], p
    occ[True] = 0  # no half-ring instantiation: a wider tile whose waiters hold at most half the CUs
    p = m.decode_plan(32)
    assert p["tp_fused"] and p["o"][0] >= 64 and not p["o_half"], p
    monkeypatch.setattr(NodeTP, "fused_row_parallel", lambda self, *a, **k: False)
    p = m.decode_plan(32)
    assert not p["tp_fused"] and not p["o_half"]


def test_tp_decode_messages_mirror_sampling_parameters():
    """The TP step protocol with decode windows: a decode / window message carries the sampling parameters
    whenever the leader's device copies changed since its last decode message (a prefill or an earlier step of
    another greedy / sampled mix rewrites them), float parameters travel as their bit patterns, and a follower's
    unpack reproduces the leader's buffers exactly; an unchanged greedy batch sends none."""
    from src.config import EngineConfig
    from src.engine.model_runner import KVPool
    from src.engine.sequence import Sequence
    from src.models.llama import CausalLM
    from src.models.presets import get_preset
    from src.parallel.tp import TPContext
    from src.parallel.tp_runner import TPModelRunner

    arch = get_preset("llama-tiny")
    runners = []
    for rank in range(2):
        tp = TPContext(rank=rank, world_size=2)
        m = CausalLM(arch, "cpu", dtype=torch.float32, tp=tp, seed=3, max_position=128)
        pool = KVPool(arch.num_layers, 16, m.hkv, 16, arch.head_dim, "cpu", dtype=torch.float32)
        r = TPModelRunner(m, pool, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, num_kv_blocks=16), 128)
        r.supports_multistep = True  # as on the GPU (windows); CPU runners default to single steps
        runners.append(r)
    lead, fol = runners
    sent = []
    lead.tp.broadcast_host = lambda t: sent.append(t.clone()) or t
    lead._bcast = lambda t: None

    def seqs(temps):
        out = []
        for i, t in enumerate(temps):
            s = Sequence(f"r{i}", [1, 2, 3], SamplingParams(max_tokens=4, temperature=t, top_k=5, top_p=0.9, seed=7 + i))
            out.append(s)
        return out

    def send(batch, pad=4):
        lead._fill_sampling(batch, pad)
        lead._sync_step(lead.KIND_DECODE, len(batch), pad)
        hdr = sent[-1].tolist()
        fol.d_pkt[: hdr[5]].copy_(lead.d_pkt[: hdr[5]])
        fol._unpack(hdr[0], hdr[1], hdr[2], hdr[4])
        return hdr

    hdr = send(seqs([0.7, 1.3, 0.0]))
    assert hdr[4] == 4  # sampled rows: parameters mirrored for the padded batch
    for name in ("d_temp", "d_topk", "d_topp", "d_seed", "d_step"):
        assert torch.equal(getattr(fol, name)[:4], getattr(lead, name)[:4]), name
    assert float(fol.d_temp[1]) == pytest.approx(1.3)
    hdr = send(seqs([0.0, 0.0, 0.0]))  # greedy after sampled: the leader rewrote them -> sent again
    assert hdr[4] == 4 and float(fol.d_temp[:4].abs().sum()) == 0.0
    hdr = send(seqs([0.0, 0.0, 0.0]))  # the same greedy batch: nothing changed, nothing sent
    assert hdr[4] == 0
