"""Disaggregated prefill → decode (two engines, KV blocks shipped) must
produce exactly the tokens a single engine produces; the wire encoding of a
KV packet must round-trip bit-exactly."""

import asyncio

import torch

from src.config import EngineConfig
from src.engine import LLMEngine
from src.engine.async_engine import AsyncLLMEngine
from src.engine.disagg import DisaggregatedServer
from src.parallel.kv_transfer import KVPacket, packet_from_wire, packet_to_wire
from src.preproc import SamplingParams

PROMPTS = [[7, 8, 9, 10] * 9, list(range(3, 50)), [400, 401]]


def eng(role_seed=5):
    cfg = EngineConfig(max_num_seqs=4, max_num_batched_tokens=128, num_kv_blocks=64, max_latency_ms=0.0)
    e = LLMEngine.from_preset("llama-tiny", device="cpu", cfg=cfg, max_model_len=256, capture=False,
                              dtype=torch.float32, seed=role_seed)
    e.eos_token_id = None
    return e


def test_disaggregated_equals_colocated():
    expect = eng().generate(PROMPTS, SamplingParams(max_tokens=7))
    srv = DisaggregatedServer(AsyncLLMEngine(eng()), AsyncLLMEngine(eng()))

    async def main():
        srv.start()
        seqs = await asyncio.wait_for(asyncio.gather(
            *(srv.generate(p, SamplingParams(max_tokens=7)) for p in PROMPTS)), 60)
        srv.stop()
        return seqs

    seqs = asyncio.run(main())
    assert [s.output_ids for s in seqs] == expect
    st = srv.stats()
    assert st["transfers"] == 3 and st["bytes_moved"] > 0
    assert st["prefill"]["kv"]["used"] == 0 and st["decode"]["kv"]["used"] == 0


def test_packet_wire_roundtrip():
    kv = torch.randn(3, 4, 64).to(torch.bfloat16)
    p = KVPacket("r", [1, 2, 3], 9, kv, 16, {"max_tokens": 4}, 12.5)
    q = packet_from_wire(packet_to_wire(p))
    assert torch.equal(q.kv.view(torch.int16), kv.view(torch.int16))
    assert (q.prompt_ids, q.first_token, q.block_size, q.ttft_ms) == ([1, 2, 3], 9, 16, 12.5)


def test_failed_prefill_still_finishes_the_overlapped_export():
    """if the forward raises after an overlapped export took its slots, the export is still finished
    (its slots get their completion event, the compute stream waits for the queued gathers) and the forward's
    exception is the one that propagates."""
    import pytest

    from src.preproc import SamplingParams

    e = eng()
    finished = []

    class FakeExporter:
        seqs = []

        def on_layer(self, li):
            pass

    e._start_export = lambda chunks: FakeExporter()
    e._finish_export = lambda ex: finished.append(ex)

    def boom(chunks, kv_hook=None):
        raise RuntimeError("forward failed")

    e.runner.prefill = boom
    e.add_request("r0", [5, 6, 7, 8], SamplingParams(max_tokens=4))
    with pytest.raises(RuntimeError, match="forward failed"):
        e.step()
    assert len(finished) == 1 and isinstance(finished[0], FakeExporter)
