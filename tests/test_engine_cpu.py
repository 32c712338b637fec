"""Engine control flow on CPU tensors (reference ops, fp32 tiny model):
continuous batching, chunked prefill, prefix caching, preemption and the
async front must not change a single greedy token."""

import asyncio
import random

import pytest
import torch

from src.config import EngineConfig
from src.engine import LLMEngine
from src.engine.async_engine import AsyncLLMEngine
from src.preproc import SamplingParams

from tests.engine_reference import greedy_reference


def make_engine(**kw):
    cfg = EngineConfig(max_num_seqs=kw.pop("max_num_seqs", 4), max_num_batched_tokens=kw.pop("budget", 64),
                       num_kv_blocks=kw.pop("blocks", 64), max_latency_ms=0.0, block_size=16,
                       enable_prefix_caching=kw.pop("prefix", True),
                       preemption_mode=kw.pop("preemption", "recompute"), swap_min_tokens=kw.pop("swap_min", 256))
    eng = LLMEngine.from_preset(kw.pop("preset", "llama-tiny"), device="cpu", cfg=cfg, max_model_len=256,
                                capture=False, dtype=torch.float32, **kw)
    eng.eos_token_id = None   # random weights may emit any id; lengths are asserted
    return eng


def prompts(n, seed=0):
    r = random.Random(seed)
    return [[r.randrange(3, 1000) for _ in range(r.randrange(5, 90))] for _ in range(n)]


def test_batched_engine_matches_no_cache_reference():
    eng = make_engine()
    ps = prompts(6)
    outs = eng.generate(ps, SamplingParams(max_tokens=5))
    for p, o in zip(ps, outs):
        assert o == greedy_reference(eng.model, p, 5)
    st = eng.get_stats()
    assert st["steps_prefill"] + st["steps_mixed"] >= 2   # budget 64 forces chunked prefill
    assert st["kv"]["used"] == 0             # every block released


def test_prefix_cache_hits_do_not_change_outputs():
    eng = make_engine()
    shared = list(range(10, 60))             # 50 tokens → 3 full blocks shared
    ps = [shared + [7, 8, 9], shared + [100, 200]]
    first = eng.generate(ps[:1], SamplingParams(max_tokens=4))
    second = eng.generate(ps[1:], SamplingParams(max_tokens=4))
    assert eng.stats["prefix_hit_tokens"] == 48
    assert first[0] == greedy_reference(eng.model, ps[0], 4)
    assert second[0] == greedy_reference(eng.model, ps[1], 4)


def test_preemption_under_kv_pressure():
    eng = make_engine(blocks=12, max_num_seqs=4, budget=256, prefix=False)
    ps = prompts(4, seed=3)
    ps = [p[:40] for p in ps]
    outs = eng.generate(ps, SamplingParams(max_tokens=30))
    assert eng.scheduler.num_preemptions > 0
    for p, o in zip(ps, outs):
        assert len(o) == 30
        assert o == greedy_reference(eng.model, p, 30)


@pytest.mark.parametrize("mode", ["swap", "auto"])
def test_swap_preemption_under_kv_pressure(mode):
    """Preempted sequences park their KV in host memory and resume without recompute
    (auto: only contexts of >= swap_min tokens swap); tokens must not change."""
    eng = make_engine(blocks=12, max_num_seqs=4, budget=256, prefix=False, preemption=mode, swap_min=48)
    ps = [p[:40] for p in prompts(4, seed=3)]
    outs = eng.generate(ps, SamplingParams(max_tokens=30))
    st = eng.get_stats()
    assert st["swaps_out"] > 0 and st["swaps_in"] == st["swaps_out"]
    assert st["swapped"] == 0 and st["kv"]["used"] == 0 and eng.scheduler.swap_used == 0
    for p, o in zip(ps, outs):
        assert o == greedy_reference(eng.model, p, 30)


@pytest.mark.parametrize("blocks,n,plen", [(6, 4, 16), (7, 5, 16), (14, 8, 32), (19, 8, 48)])
def test_swap_in_and_lockstep_block_crossing(blocks, n, plen):
    """Lockstep sequences (equal prompt lengths) all need a new KV block in the same step as a
    swapped sequence resumes: the resumed sequence must not be re-swapped with its
    fresh, unfilled blocks, and no KV may be lost — tokens equal the no-cache reference."""
    # (configurations found to crash the round-1 scheduler with AttributeError on swap_buf = None)
    eng = make_engine(blocks=blocks, max_num_seqs=n, budget=512, prefix=False, preemption="swap", swap_min=0)
    r = random.Random(1)
    ps = [[r.randrange(3, 1000) for _ in range(plen)] for _ in range(n)]  # lockstep
    outs = eng.generate(ps, SamplingParams(max_tokens=40))
    st = eng.get_stats()
    assert st["swaps_out"] > 0 and st["swaps_in"] == st["swaps_out"]
    assert st["kv"]["used"] == 0 and eng.scheduler.swap_used == 0
    for p, o in zip(ps, outs):
        assert o == greedy_reference(eng.model, p, 40)


def test_resumed_sequence_is_last_resort_victim():
    from src.engine.sequence import Sequence, SeqStatus
    from src.preproc import SamplingParams as SP

    eng = make_engine(blocks=16, max_num_seqs=4)
    sch = eng.scheduler
    a = Sequence("a", [1, 2, 3], SP(max_tokens=4))
    b = Sequence("b", [1, 2, 3], SP(max_tokens=4))
    a.arrival, b.arrival = 1.0, 2.0
    for q in (a, b):
        q.status = SeqStatus.RUNNING
        sch.running.append(q)
    sch._resumed_now = {id(b)}           # b (newest) was swapped back in this step
    c = Sequence("c", [1], SP(max_tokens=1))
    assert sch._pick_victim(exclude=c) is a
    sch._resumed_now = set()
    assert sch._pick_victim(exclude=c) is b


def test_swap_abort_releases_swap_space():
    eng = make_engine(blocks=12, max_num_seqs=4, budget=256, prefix=False, preemption="swap")
    for i, p in enumerate(prompts(4, seed=3)):
        eng.add_request(f"r{i}", p[:40], SamplingParams(max_tokens=30))
    while not eng.scheduler.swapped:
        eng.step()
    victim = eng.scheduler.swapped[0]
    eng.abort(victim.request_id)
    assert eng.scheduler.swap_used == 0 or eng.scheduler.swapped
    while eng.has_work():
        eng.step()
    assert eng.scheduler.swap_used == 0 and eng.get_stats()["kv"]["used"] == 0


def test_moe_engine():
    eng = make_engine(preset="mixtral-tiny")
    ps = prompts(3, seed=5)
    outs = eng.generate(ps, SamplingParams(max_tokens=4))
    for p, o in zip(ps, outs):
        assert o == greedy_reference(eng.model, p, 4)


def test_stop_conditions_and_validation():
    eng = make_engine()
    eng.eos_token_id = None
    sp = SamplingParams(max_tokens=8)
    first = eng.generate([[5, 6, 7]], sp)[0]
    stop_tok = first[2]
    got = eng.generate([[5, 6, 7]], SamplingParams(max_tokens=8, stop_token_ids=[stop_tok]))[0]
    assert got == first[:3]
    with pytest.raises(ValueError):
        eng.add_request("x", list(range(300)), SamplingParams(max_tokens=1))


def test_async_engine_concurrent_requests():
    eng = make_engine()
    ae = AsyncLLMEngine(eng)
    ps = prompts(5, seed=9)

    async def main():
        ae.start()
        futs = [ae.submit(f"r{i}", p, SamplingParams(max_tokens=4)) for i, p in enumerate(ps)]
        seqs = await asyncio.wait_for(asyncio.gather(*futs), 60)
        ae.stop()
        return seqs

    seqs = asyncio.run(main())
    for p, s in zip(ps, seqs):
        assert s.output_ids == greedy_reference(eng.model, p, 4)
        assert s.ttft_ms() is not None and s.latency_ms() >= s.ttft_ms()


def test_sampled_generation_is_seeded():
    eng = make_engine()
    sp = SamplingParams(max_tokens=6, temperature=1.0, top_k=20, top_p=0.9, seed=123)
    a = eng.generate([[4, 5, 6]], sp)[0]
    b = eng.generate([[4, 5, 6]], sp)[0]
    assert a == b and len(a) == 6


def test_reference_copy_is_an_fp32_twin():
    """CausalLM.reference_copy (the fp32 oracle of tests/test_oracle_gpu.py): same weights in fp32,
    independent tensors, same greedy tokens as the source model on the reference ops."""
    import sys

    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_oracle_gpu import paged_greedy

    from src.models.llama import CausalLM
    from src.models.presets import get_preset

    m = CausalLM(get_preset("llama-tiny"), "cpu", dtype=torch.bfloat16, seed=1, max_position=512)
    r = m.reference_copy("cpu", torch.float32)
    assert r.layers[0].qkv.dtype == torch.float32 and r.layers[0].qkv.data_ptr() != m.layers[0].qkv.data_ptr()
    assert torch.equal(r.layers[1].down.to(torch.bfloat16), m.layers[1].down)
    ps = [[5, 9, 33, 12, 7] * 4, [100, 200, 300]]
    a, b = paged_greedy(m, ps, 4), paged_greedy(r, ps, 4)
    assert float((a[2][0] - b[2][0]).norm() / b[2][0].norm()) < 0.02


def test_mixed_steps_admit_prompts_while_decoding():
    """Requests arriving while others decode ride along in mixed steps (decode rows + prompt chunks of
    at most mixed_step_tokens rows in ONE ragged batch): no prefill-only step stalls the running
    sequences, long prompts are chunked across several mixed steps, and no greedy token changes."""
    eng = make_engine(max_num_seqs=6, budget=256, blocks=128)
    eng.cfg.mixed_step_tokens = 24
    eng.cfg.mixed_batching = "always"
    ps = prompts(6, seed=11)
    sp = SamplingParams(max_tokens=12)
    got = {}
    for i in range(2):
        eng.add_request(f"a{i}", ps[i], sp, on_finish=lambda s, i=i: got.__setitem__(i, list(s.output_ids)))
    eng.step()  # the first two prompts: a plain prefill step (nothing is decoding yet)
    assert eng.scheduler.steps_prefill == 1
    step = 0
    while eng.has_work():
        if step < 4:  # one arrival per step while the first two decode
            j = 2 + step
            eng.add_request(f"a{j}", ps[j], sp, on_finish=lambda s, j=j: got.__setitem__(j, list(s.output_ids)))
        n_dec = len([s for s in eng.scheduler.running if not s.in_prefill])
        eng.step()
        step += 1
        assert n_dec == 0 or eng.scheduler.steps_prefill == 1  # never a prefill-only step while decoding
    st = eng.get_stats()
    assert st["steps_mixed"] >= 4 and st["kv"]["used"] == 0
    for i, p in enumerate(ps):
        assert got[i] == greedy_reference(eng.model, p, 12), i


def test_mixed_batching_off_keeps_prefill_only_steps():
    eng = make_engine(max_num_seqs=4, budget=256)
    eng.cfg.mixed_batching = "off"
    ps = prompts(3, seed=12)
    sp = SamplingParams(max_tokens=6)
    eng.add_request("x0", ps[0], sp)
    eng.step()
    eng.step()  # decoding
    eng.add_request("x1", ps[1], sp)
    eng.step()
    assert eng.scheduler.steps_mixed == 0 and eng.scheduler.steps_prefill == 2


def test_mixed_auto_policy():
    """auto: a short prompt arriving while others decode rides along in a mixed step; a long one gets a
    bounded prefill step (prefill_tokens_while_decoding) and the very next step decodes again."""
    eng = make_engine(max_num_seqs=6, budget=256, blocks=128)
    eng.cfg.mixed_step_tokens = 16
    eng.cfg.prefill_tokens_while_decoding = 48
    sp = SamplingParams(max_tokens=10)
    long_p, short_p = prompts(1, seed=20)[0][:5] * 20, [5, 6, 7, 8]
    got = {}
    eng.add_request("d0", [9, 10, 11, 12, 13], sp, on_finish=lambda s: got.__setitem__(0, list(s.output_ids)))
    eng.step()
    eng.step()
    s0 = dict(eng.scheduler.stats())
    eng.add_request("short", short_p, sp, on_finish=lambda s: got.__setitem__(1, list(s.output_ids)))
    eng.step()
    assert eng.scheduler.steps_mixed == s0["steps_mixed"] + 1       # 1 decode row + 4 prompt rows <= 16
    eng.add_request("long", long_p, sp, on_finish=lambda s: got.__setitem__(2, list(s.output_ids)))
    kinds = []
    while eng.has_work():
        st = dict(eng.scheduler.stats())
        eng.step()
        d = {k: eng.scheduler.stats()[k] - st[k] for k in ("steps_prefill", "steps_decode", "steps_mixed")}
        kinds.append(max(d, key=d.get))
    assert kinds[0] == "steps_prefill"                               # 100 tokens > 16 spare rows: bounded step
    assert all(not (a == b == "steps_prefill") for a, b in zip(kinds, kinds[1:]))  # never two stalls in a row
    for i, p in enumerate(([9, 10, 11, 12, 13], short_p, long_p)):
        assert got[i] == greedy_reference(eng.model, p, 10), i


def test_prefill_batching_under_load():
    """prefill_batch_tokens: while a sequence decodes, a prompt needing a prefill step is held (decode
    steps continue) until enough prompt tokens wait or the oldest has waited prefill_batch_wait_ms."""
    eng = make_engine(max_num_seqs=6, budget=256, blocks=128)
    eng.cfg.mixed_batching = "off"
    eng.cfg.prefill_batch_tokens = 60
    eng.cfg.prefill_batch_wait_ms = 1e6
    sp = SamplingParams(max_tokens=12)
    got = {}
    ps = [p[:5] * 5 for p in prompts(3, seed=21)]  # 25-token prompts
    eng.add_request("d0", [9, 10, 11, 12, 13], sp, on_finish=lambda s: got.__setitem__(0, list(s.output_ids)))
    eng.step()
    eng.add_request("a", ps[0], sp, on_finish=lambda s: got.__setitem__(1, list(s.output_ids)))
    st = dict(eng.scheduler.stats())
    eng.step()
    eng.step()
    assert eng.scheduler.stats()["steps_prefill"] == st["steps_prefill"]     # 25 < 60 tokens: held
    assert eng.scheduler.defer_deadline is not None
    eng.add_request("b", ps[1], sp, on_finish=lambda s: got.__setitem__(2, list(s.output_ids)))
    eng.step()
    assert eng.scheduler.stats()["steps_prefill"] == st["steps_prefill"]     # 50 < 60: still held
    eng.add_request("c", ps[2], sp, on_finish=lambda s: got.__setitem__(3, list(s.output_ids)))
    eng.step()
    assert eng.scheduler.stats()["steps_prefill"] == st["steps_prefill"] + 1  # 75 >= 60: one prefill step
    eng.cfg.prefill_batch_wait_ms = 0.0                                       # deadline passed: admit at once
    eng.add_request("e", ps[0][:7], sp, on_finish=lambda s: got.__setitem__(4, list(s.output_ids)))
    st = dict(eng.scheduler.stats())
    eng.step()
    assert eng.scheduler.stats()["steps_prefill"] == st["steps_prefill"] + 1
    while eng.has_work():
        eng.step()
    for i, p in enumerate(([9, 10, 11, 12, 13], ps[0], ps[1], ps[2], ps[0][:7])):
        assert got[i] == greedy_reference(eng.model, p, 12), i


def test_always_mixed_does_not_starve_prompts_behind_a_large_decode_batch():
    """mixed_batching="always" with at least mixed_step_tokens decoding sequences used to leave a
    budget of 0 rows for prompt chunks: a new arrival (or a running chunked prefill) made no progress
    until enough decoders finished. It now falls back to the prefill/decode alternation."""
    eng = make_engine(max_num_seqs=12, budget=256, blocks=256)
    eng.cfg.mixed_step_tokens = 8
    eng.cfg.mixed_batching = "always"
    ps = prompts(11, seed=21)
    long_sp, short_sp = SamplingParams(max_tokens=40), SamplingParams(max_tokens=4)
    got = {}
    for i in range(10):  # 10 decoders > mixed_step_tokens
        eng.add_request(f"d{i}", ps[i][:20], long_sp)
    eng.step()
    eng.step()
    eng.add_request("late", ps[10], short_sp, on_finish=lambda s: got.__setitem__("late", list(s.output_ids)))
    for _ in range(12):  # well before any of the 40-token decoders can finish
        eng.step()
        if "late" in got:
            break
    assert "late" in got, "the late prompt was starved by the decode batch"
    assert got["late"] == greedy_reference(eng.model, ps[10], 4)
    while eng.has_work():
        eng.step()
    assert eng.get_stats()["kv"]["used"] == 0


def test_lm_head_argmax_candidates_are_never_left_stale():
    """compute_logits(argmax_parts=...) promises per-tile greedy candidates that the sampler reads instead of the
    logits; a head that cannot write them (row-major here: not in tile order) must refuse loudly, and it reports
    zero candidate tiles so the runner never asks."""
    from src.models.llama import CausalLM
    from src.models.presets import get_preset

    m = CausalLM(get_preset("llama-tiny"), "cpu", dtype=torch.float32, seed=1, max_position=256)
    assert m.lm_head_argmax_parts() == 0
    h = torch.randn(4, m.arch.hidden_size)
    with pytest.raises(ValueError):
        m.compute_logits(h, argmax_parts=torch.zeros(4, 8, 2, dtype=torch.int32))
    assert m.compute_logits(h).shape == (4, m.arch.vocab_size)


def test_decode_weight_layout_choice(monkeypatch):
    """EngineConfig.decode_weight_layout: "auto" drops the tile-order decode weight copies when
    the KV pool is the constraint — kv_capacity_priority (config 5), or an explicit num_kv_blocks the HBM left
    after the copies cannot hold — and keeps them otherwise; explicit layouts win; the engine reports its choice."""
    import src.engine.llm_engine as le
    from src.config import EngineConfig
    from src.models.presets import get_preset

    class M:
        arch = get_preset("llama3-8b")
        hkv = 8

        def decode_copy_bytes(self, buckets):
            return 13 << 30

    per_block = le.KVPool.bytes_per_block(32, 8, 16, 128)  # 2 MiB
    monkeypatch.setattr(le, "plan_kv_blocks", lambda arch, model, cfg, dev: 100000)
    cuda = torch.device("cuda")
    choose = le.choose_decode_weight_layout
    assert choose(M(), EngineConfig(), cuda, [32]) == "tiled"
    assert choose(M(), EngineConfig(kv_capacity_priority=True), cuda, [32]) == "single"
    assert choose(M(), EngineConfig(kv_capacity_priority=True, decode_weight_layout="tiled"), cuda, [32]) == "tiled"
    assert choose(M(), EngineConfig(decode_weight_layout="single"), cuda, [32]) == "single"
    room = 100000 - (13 << 30) // per_block
    assert choose(M(), EngineConfig(num_kv_blocks=room), cuda, [32]) == "tiled"
    assert choose(M(), EngineConfig(num_kv_blocks=room + 1), cuda, [32]) == "single"
    with pytest.raises(ValueError):
        choose(M(), EngineConfig(decode_weight_layout="bogus"), cuda, [32])
    eng = LLMEngine.from_preset("llama-tiny", device="cpu", cfg=EngineConfig(num_kv_blocks=64), max_model_len=128)
    assert eng.get_stats()["decode_weight_layout"] == "row-major"  # no tile-order copies off the GPU
