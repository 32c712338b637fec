"""Queued decode windows (EngineConfig.async_decode) — the engine-side protocol, on CPU.

A deterministic fake runner stands in for the GPU one: the token a sequence samples at position p is
a pure function of (its prompt, p), and a "queued" window is computed when it is queued but handed
back only by the next ``decode_continue``, exactly like the device. The engine must produce the same
outputs with and without queued windows (mixed lengths, stop tokens inside a queued window, late
arrivals, aborts) and must not leak KV blocks. The GPU counterpart with the real runner is
tests/test_engine_gpu.py::test_queued_decode_windows_match_synchronous."""

import random

import torch

from src.config import EngineConfig
from src.engine import LLMEngine
from src.engine.model_runner import ModelRunner
from src.preproc import SamplingParams


def tok_at(seq, pos):
    h = hash((tuple(seq.prompt_ids[:8]), len(seq.prompt_ids), pos))
    return 3 + h % 997


class FakeRunner(ModelRunner):
    """Host-only runner with the multi-step / queued-window interface of ModelRunner."""

    def __init__(self, model, pool, cfg, max_model_len):
        super().__init__(model, pool, cfg, max_model_len)
        self.supports_multistep = True
        self.queued = 0

    def capture_graphs(self):
        pass

    def prefill(self, chunks):
        out = []
        for c in chunks:  # the token after the chunk's last position (a decode row, a whole or recomputed prompt)
            out.append(tok_at(c.seq, c.start + c.length) if (c.decode or c.completes_prompt) else None)
        return out

    def decode(self, seqs):
        return [tok_at(s, len(s)) for s in seqs]

    def _window(self, seqs, pending, k):
        return [[tok_at(s, len(s) + pending + i) for s in seqs] for i in range(k)]

    def decode_multi(self, seqs, k, k_next=0):
        assert self.inflight is None
        for s in seqs:  # the caller reserved slots for both windows
            assert len(s.block_table) * self.bs >= len(s) + k - 1
        toks = self._window(seqs, 0, k)
        if k_next > 1:
            self._queue(seqs, k, k_next)
        return toks

    def _queue(self, seqs, pending, k):
        for s in seqs:
            assert len(s.block_table) * self.bs >= len(s) + pending + k - 1, "slots not reserved"
        self.inflight = {"seqs": list(seqs), "k": k, "toks": self._window(seqs, pending, k)}
        self.queued += 1

    def decode_continue(self, k_next=0):
        w = self.inflight
        self.inflight = None
        if k_next > 1:
            self._queue(w["seqs"], w["k"], k_next)
        return w["toks"]


def make_engine(async_decode, blocks=256, window=4):
    cfg = EngineConfig(max_num_seqs=8, max_num_batched_tokens=512, num_kv_blocks=blocks, max_latency_ms=0.0,
                       block_size=16, decode_window=window, async_decode=async_decode,
                       preemption_mode="recompute")
    eng = LLMEngine.from_preset("llama-tiny", device="cpu", cfg=cfg, max_model_len=256, capture=False,
                                dtype=torch.float32)
    eng.runner = FakeRunner(eng.model, eng.pool, cfg, eng.max_model_len)
    eng.eos_token_id = None
    return eng


def run(eng, reqs, late=None, late_at=3, abort_at=None):
    res = {}

    def add(i, p, sp):
        eng.add_request(f"r{i}", p, sp, on_finish=lambda s, i=i: res.__setitem__(i, list(s.output_ids)))

    for i, (p, sp) in enumerate(reqs):
        add(i, p, sp)
    steps = 0
    while eng.has_work():
        eng.step()
        steps += 1
        if late is not None and steps == late_at:
            add(len(reqs), *late)
        if abort_at is not None and steps == abort_at:
            eng.abort("r1")
    return res


def reqs_for(seed=0, stop_on=None):
    r = random.Random(seed)
    ps = [[r.randrange(3, 1000) for _ in range(r.randrange(5, 60))] for _ in range(6)]
    lens = [30, 9, 41, 17, 25, 33]
    out = []
    for i, (p, n) in enumerate(zip(ps, lens)):
        out.append((p, SamplingParams(max_tokens=n, stop_token_ids=[stop_on] if (stop_on and i == 0) else [])))
    return out


def test_queued_windows_same_tokens_as_synchronous():
    a, b = make_engine(False), make_engine(True)
    ra, rb = run(a, reqs_for()), run(b, reqs_for())
    assert ra == rb
    assert b.runner.queued > 0 and b.stats.get("queued_windows", 0) > 0
    assert a.runner.queued == 0
    assert a.blocks.bm.num_available() == b.blocks.bm.num_available()
    assert all(len(v) == n for v, (_, sp) in zip([rb[i] for i in range(6)], reqs_for())
               for n in [sp.max_tokens])


def test_stop_token_inside_a_queued_window():
    base = run(make_engine(False), reqs_for())
    stop = base[0][20]
    first = base[0].index(stop)
    a, b = make_engine(False), make_engine(True)
    ra, rb = run(a, reqs_for(stop_on=stop)), run(b, reqs_for(stop_on=stop))
    assert ra == rb and len(rb[0]) == first + 1
    assert a.blocks.bm.num_available() == b.blocks.bm.num_available()


def test_late_arrival_and_abort_end_the_chain():
    late = ([5, 6, 7, 8, 9, 10, 11], SamplingParams(max_tokens=12))
    a, b = make_engine(False), make_engine(True)
    ra = run(a, reqs_for(), late=late, late_at=4, abort_at=6)
    rb = run(b, reqs_for(), late=late, late_at=4, abort_at=6)
    assert set(ra) == set(rb) == set(range(7))
    for i in ra:
        if i != 1:  # the aborted request may stop at a different token (windows differ in length)
            assert ra[i] == rb[i], i
    assert rb[1] == ra[1][: len(rb[1])] or ra[1] == rb[1][: len(ra[1])]
    assert a.blocks.bm.num_available() == b.blocks.bm.num_available()
    assert not b.has_work() and b.runner.inflight is None


def test_no_queued_window_when_blocks_run_short():
    # a pool too small to reserve two windows ahead for everyone: the engine falls back to synchronous
    # windows (or single steps) and still finishes every request with the same tokens
    a, b = make_engine(False, blocks=40), make_engine(True, blocks=40)
    ra, rb = run(a, reqs_for()), run(b, reqs_for())
    assert ra == rb


def test_open_loop_arrivals_stop_queued_continuations_but_not_closed_loop_waves():
    """Requests arriving while sequences decode (open-loop traffic) stop the engine from queueing a continuation
    window behind the running one, so the next arrival waits for at most one window; a closed-loop wave (its
    requests arrive while the engine is idle) never counts. Tokens are unchanged either way."""
    import time

    eng = make_engine(True)
    base = run(make_engine(True), reqs_for())
    reqs = reqs_for()
    for i, (p, sp) in enumerate(reqs):  # idle engine: a closed-loop wave
        eng.add_request(f"r{i}", p, sp)
    assert len(eng._dec_arrivals) == 0 and eng._arrival_cap(continuation=True) > 1
    eng.step()  # prefill: the wave is running now
    late = [[5 + i, 6, 7, 8, 9] for i in range(2)]
    for j, p in enumerate(late):  # two open-loop arrivals while decoding
        eng.add_request(f"late{j}", p, SamplingParams(max_tokens=3))
    assert len(eng._dec_arrivals) == 2
    assert eng._arrival_cap(continuation=True) == 0 and eng._arrival_cap() > 1  # noqueue: only continuations
    eng._dec_arrivals.clear()
    eng._dec_arrivals.extend([time.perf_counter() - 10.0] * 2)  # older than the lookback: no effect
    assert eng._arrival_cap(continuation=True) > 1
    res = {}
    eng2 = make_engine(True)
    for i, (p, sp) in enumerate(reqs):
        eng2.add_request(f"r{i}", p, sp, on_finish=lambda s, i=i: res.__setitem__(i, list(s.output_ids)))
    steps = 0
    while eng2.has_work():
        eng2.step()
        steps += 1
        if steps in (2, 3):
            eng2.add_request(f"x{steps}", [3, 4, 5, 6], SamplingParams(max_tokens=4))
    assert res == base  # the policy changes when windows run, not what they compute
