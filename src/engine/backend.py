"""
LLMBackend: the worker-side model session for ``arch in {"llama","mixtral"}``
(the GPU replacement of the reference's ``FakeModel``,
`/root/reference/src/mock_models/fake_model.py:33-67`).

``predict(inputs)`` accepts the LLM request format documented in
:func:`src.preproc.normalize_request` and returns
``{"token_ids", "text", "num_prompt_tokens", "num_output_tokens",
"finish_reason", "ttft_ms", "latency_ms", "tpot_ms"}``.
"""

from __future__ import annotations

import asyncio
import logging
import os
import time
import uuid
from typing import Any, Dict, List, Optional

import torch

from src.config import EngineConfig, ModelConfig
from src.engine.async_engine import AsyncLLMEngine
from src.engine.llm_engine import LLMEngine
from src.postproc import build_llm_output
from src.preproc import ByteTokenizer, load_tokenizer, normalize_request

logger = logging.getLogger(__name__)

_DEFAULT_PRESET = {"llama": "llama3-8b", "mixtral": "mixtral-8x7b"}


def engine_config_from(config: ModelConfig) -> EngineConfig:
    ov = config.overrides or {}
    return EngineConfig(
        max_num_seqs=config.max_batch_size,
        max_num_batched_tokens=config.max_num_batched_tokens,
        max_latency_ms=config.max_latency_ms,
        block_size=config.kv_block_size,
        num_kv_blocks=config.num_kv_blocks,
        gpu_memory_fraction=config.gpu_memory_fraction,
        enable_prefix_caching=config.enable_prefix_caching,
        kv_block_ttl_s=ov.get("kv_block_ttl_s"),
        use_cuda_graph=config.use_cuda_graph,
        kv_capacity_priority=bool(ov.get("kv_capacity_priority", False)),
        decode_weight_layout=str(ov.get("decode_weight_layout", "auto")),
    )


class LLMBackend:
    def __init__(self, config: ModelConfig, engine: Optional[LLMEngine] = None):
        self.config = config
        preset = config.preset or _DEFAULT_PRESET[config.arch]
        device = config.overrides.get("device") if config.overrides else None
        if device is None:
            device = "cuda:0" if torch.cuda.is_available() else "cpu"
        if str(device).startswith("cuda") and torch.device(device).index is not None:
            # model build, weight packing and graph capture run on this thread: on the serving GPU
            torch.cuda.set_device(torch.device(device))
        if engine is None:
            from src.models.loader import is_hf_checkpoint

            ecfg = engine_config_from(config)
            if is_hf_checkpoint(config.model_path):  # real weights from a local checkpoint directory
                engine = LLMEngine.from_pretrained(config.model_path, device=device, cfg=ecfg,
                                                   max_model_len=config.max_model_len,
                                                   capture=config.use_cuda_graph)
            else:
                engine = LLMEngine.from_preset(preset, device=device, cfg=ecfg, max_model_len=config.max_model_len,
                                               seed=config.seed, capture=config.use_cuda_graph)
        self.engine = engine
        self.tokenizer = load_tokenizer(config.model_path or None, engine.arch.vocab_size)
        if not isinstance(self.tokenizer, ByteTokenizer):
            engine.eos_token_id = getattr(self.tokenizer, "eos_token_id", engine.eos_token_id)
        self.async_engine = AsyncLLMEngine(engine, name=config.model_name)
        self.role = config.role
        self._decode_link = None
        if self.role == "prefill":
            from src.engine.disagg import RemoteDecodeLink

            addr = (config.overrides or {}).get("decode_worker")
            if addr:
                self._decode_link = RemoteDecodeLink(addr, config.model_name)
        self.request_count = 0
        self.error_count = 0
        self.total_latency = 0.0
        self._live: Dict[str, str] = {}  # client request_id -> engine request id (abort)
        self._zone = None                # IPC landing zone for shipped KV (decode role, lazily)
        ov = config.overrides or {}
        # prefill role: gather each prompt's KV straight into a slot of the decode worker's landing zone reserved
        # before the prompt runs (False: gather locally, then copy into a slot — the staged path, A/B only)
        self.kv_direct = bool(ov.get("kv_direct", True))
        self.kv_zone_bytes = int(ov.get("kv_landing_zone_bytes", 4 << 30))
        self.ipc_imports = 0
        # text prompts and text outputs tokenised / detokenised in separate processes (ModelConfig.preproc_processes;
        # the reference's "pre/post-processing in a separate process", /root/reference/README.md:15,96-98). Token-id
        # requests (the benches' path) never touch the pool; streaming deltas stay incremental on the event loop.
        self.preproc = None
        nproc = int(getattr(config, "preproc_processes", 0) or ov.get("preproc_processes", 0) or 0)
        if nproc > 0:
            from src.preproc import PreprocPool

            tok_path = None if isinstance(self.tokenizer, ByteTokenizer) else (config.model_path or None)
            self.preproc = PreprocPool(nproc, engine.arch.vocab_size, tok_path)

    async def start(self) -> None:
        self.async_engine.start()

    async def stop(self) -> None:
        self.async_engine.stop()

    def close(self) -> None:
        self.async_engine.stop()
        if self.preproc is not None:
            self.preproc.close()
            self.preproc = None

    async def _tokenized(self, inputs: Any) -> Any:
        """A text prompt's ids from the pre-processing pool (unchanged inputs without a pool or with ids)."""
        if self.preproc is None:
            return inputs
        if isinstance(inputs, str):
            inputs = {"prompt": inputs}
        if isinstance(inputs, dict) and inputs.get("prompt_token_ids") is None and isinstance(inputs.get("prompt"), str):
            ids = await self.preproc.encode_one(inputs["prompt"])
            inputs = {**inputs, "prompt_token_ids": ids}
        return inputs

    async def _output(self, ids: List[int], return_text: bool = True, **kw) -> Dict[str, Any]:
        """build_llm_output, with the text detokenised in the post-processing pool when there is one."""
        if self.preproc is None or not return_text:
            return build_llm_output(ids, self.tokenizer, return_text=return_text, **kw)
        out = build_llm_output(ids, None, return_text=False, **kw)
        out["text"] = await self.preproc.decode_one(ids)
        return out

    def healthy(self) -> bool:
        """False once the engine loop died (e.g. a HIP fault surfaced as an exception): the worker
        then reports itself unhealthy and fails requests as retryable elsewhere."""
        return self.async_engine.error is None

    def load(self) -> float:
        s = self.engine.scheduler
        return (len(s.running) + len(s.waiting)) / max(1, self.engine.cfg.max_num_seqs)

    def load_report(self) -> Dict[str, Any]:
        """Engine state for the load balancer (piggybacked on every reply and health answer by the worker): the
        engine thread's last snapshot, plus the submissions its loop has not drained yet."""
        r = dict(self.engine.load_snapshot)
        if not r:
            r = {"running": 0, "waiting": 0, "waiting_prompt_tokens": 0, "max_num_seqs": self.engine.cfg.max_num_seqs,
                 "kv_used_frac": 0.0, "step_ms": round(self.engine._step_est * 1e3, 4), "prefill_us_per_token": 0.0}
        r["waiting"] = r.get("waiting", 0) + self.async_engine._q.qsize()
        return r

    async def predict(self, inputs: Any, request_id: Optional[str] = None,
                      on_token=None) -> Dict[str, Any]:
        """One generation. ``inputs["timeout_s"]`` bounds it (the request is aborted in the engine and the
        tokens so far come back with ``finish_reason="timeout"``); a cancelled caller (client gone) aborts
        it too, so an abandoned request never keeps its batch slot and KV blocks. ``request_id`` names it
        for :meth:`abort_request`; ``on_token(tok)`` streams tokens (event-loop thread)."""
        if not self.async_engine.running:
            self.async_engine.start()
        self.request_count += 1
        try:
            inputs = await self._tokenized(inputs)
            gi = normalize_request(inputs, self.tokenizer, self.engine.max_model_len)
        except ValueError:
            self.error_count += 1
            raise
        rid = uuid.uuid4().hex
        t0 = time.perf_counter()
        if self._decode_link is not None and gi.sampling.max_tokens > 1:
            return await self._prefill_then_ship(rid, gi, t0)
        timeout = inputs.get("timeout_s") if isinstance(inputs, dict) else None
        if request_id:
            self._live[request_id] = rid
        fut = self.async_engine.submit(rid, gi.prompt_token_ids, gi.sampling, on_token=on_token)
        timed_out = False
        try:
            if timeout:
                try:
                    seq = await asyncio.wait_for(asyncio.shield(fut), float(timeout))
                except asyncio.TimeoutError:
                    timed_out = True
                    self.async_engine.abort(rid)
                    seq = await fut
            else:
                seq = await fut
        except asyncio.CancelledError:
            self.async_engine.abort(rid)
            raise
        finally:
            if request_id:
                self._live.pop(request_id, None)
        lat = (time.perf_counter() - t0) * 1e3
        self.total_latency += lat / 1e3
        reason = "timeout" if timed_out and seq.finish_reason == "abort" else (seq.finish_reason or "length")
        return await self._output(seq.output_ids, gi.return_text, prompt_len=seq.prompt_len, finish_reason=reason,
                                  ttft_ms=seq.ttft_ms(), latency_ms=seq.latency_ms())

    async def predict_stream(self, inputs: Any, emit, request_id: Optional[str] = None) -> Dict[str, Any]:
        """Streaming generation: ``await emit({"delta_token_ids": [...], "done": False})`` as tokens are
        produced, then return the final output. If ``emit`` fails (client gone) the request is aborted.

        The first token (the prefill's) always goes out ALONE, as soon as it reaches the event loop — TTFT
        is what a streaming client is for, and it must not depend on how far the engine thread has run
        ahead (a small model can finish the whole generation before this coroutine first wakes: coalescing
        everything queued would then send one frame for the whole request). Later tokens are coalesced per
        wake-up (bursts of up to ``decode_window`` per host round trip)."""
        q: asyncio.Queue = asyncio.Queue()
        task = asyncio.ensure_future(self.predict(inputs, request_id, on_token=q.put_nowait))
        with_text = not isinstance(inputs, dict) or bool(inputs.get("return_text", True))
        so_far: List[int] = []
        text_sent = 0
        first = True

        async def send(toks: List[int]) -> None:
            nonlocal text_sent
            frame: Dict[str, Any] = {"delta_token_ids": toks, "done": False}
            so_far.extend(toks)
            if with_text:  # incremental detokenisation: hold back a trailing partial character
                text = self.tokenizer.decode(so_far)
                if text.endswith("\ufffd"):
                    text = text.rstrip("\ufffd")
                frame["delta_text"] = text[text_sent:]
                text_sent = max(text_sent, len(text))
            await emit(frame)

        try:
            while True:
                get = asyncio.ensure_future(q.get())
                done, _ = await asyncio.wait({get, task}, return_when=asyncio.FIRST_COMPLETED)
                if get not in done:
                    get.cancel()
                    break
                toks = [get.result()]
                while not first and not q.empty():
                    toks.append(q.get_nowait())
                first = False
                await send(toks)
            toks = []
            while not q.empty():  # tokens delivered before the completion callback ran
                toks.append(q.get_nowait())
            if toks:
                await send(toks)
            out = await task
            if with_text and isinstance(out.get("text"), str) and len(out["text"]) > text_sent:
                await emit({"delta_token_ids": [], "delta_text": out["text"][text_sent:], "done": False})
            return out
        except BaseException:
            task.cancel()
            raise

    def abort_request(self, request_id: str) -> bool:
        rid = self._live.get(request_id)
        if rid is None:
            return False
        self.async_engine.abort(rid)
        return True

    async def _prefill_then_ship(self, rid: str, gi, t0: float) -> Dict[str, Any]:
        from src.engine.disagg import sampling_to_dict
        from src.parallel.kv_transfer import KVPacket

        # try to reserve the decode worker's landing-zone slot first (no waiting: a full zone must not hold the
        # prompt out of the prefill queue): the prefill engine's export then gathers the prompt's blocks
        # straight into it (one pass over xGMI, no staging tensor, no second copy). Otherwise the packet takes
        # the staged path, whose reserve may wait for space AFTER the prompt has run.
        slot = None
        if self.engine.device.type == "cuda" and self.kv_direct:
            from src.parallel.kv_transfer import packet_shape

            nb = self.engine.blocks.blocks_needed(len(gi.prompt_token_ids))
            slot = await self._decode_link.reserve_export(self.engine.device,
                                                          packet_shape(self.engine.pool.planes(), nb))
        ud = {"export_kv": True}
        if slot is not None:
            ud["export_slot"] = slot
        try:
            pseq = await self.async_engine.submit(rid, gi.prompt_token_ids, gi.sampling, user_data=ud)
        except BaseException:
            # a cancelled await does not stop the prompt by itself: abort it, and give the slot back as soon as
            # no gather can still write into it (at once if none was queued, else behind its event)
            self.async_engine.abort(rid)
            if slot is not None:
                self._decode_link.revoke(slot)
            raise
        if slot is not None and slot.state != "taken":  # past the reservation's deadline: staged path
            self._decode_link.revoke(slot)
            slot = None
        if pseq.finish_reason == "stop":
            if slot is not None:
                self._decode_link.revoke(slot)
            return await self._output(pseq.output_ids, gi.return_text, prompt_len=pseq.prompt_len,
                                      finish_reason="stop", ttft_ms=pseq.ttft_ms(), latency_ms=pseq.latency_ms())
        packet = KVPacket(rid, gi.prompt_token_ids, pseq.output_ids[0], pseq.kv_export, self.engine.cfg.block_size,
                          sampling_to_dict(gi.sampling), ttft_ms=pseq.ttft_ms(),
                          ready=getattr(pseq, "kv_export_ready", None))
        pseq.kv_export = None
        if slot is not None:
            rep = await self._decode_link.send_reserved(packet, slot.res)
        else:
            rep = await self._decode_link.send(packet)
        if not rep.get("success"):
            raise RuntimeError(f"decode worker failed: {rep.get('error')}")
        out = rep["outputs"]
        out["latency_ms"] = (time.perf_counter() - t0) * 1e3
        out["disaggregated"] = True
        return out

    def _landing_zone(self):
        if self._zone is None:
            from src.parallel.kv_transfer import IPCLandingZone

            # uncached (fine-grained) segments: a peer GPU's stores over xGMI are not cached in this GPU's L2
            # under a stale line (coherence; no measurable cost, profiles/r4_disagg_zone_uncached_vs_cached.jsonl)
            self._zone = IPCLandingZone(self.engine.device, self.kv_zone_bytes, uncached=True)
        return self._zone

    async def _kv_import(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        from src.engine.disagg import packet_for_import
        from src.parallel.kv_transfer import KVPacket
        from src.preproc import SamplingParams

        d = msg["packet"]
        handed: List[bool] = []
        off = -1
        ready = None
        if d.get("ipc") is not None:  # payload delivered (or being delivered) into the landing zone by the sender
            zone, off = self._landing_zone(), int(d["ipc"]["offset"])
            kv = zone.claim(off, d["shape"], d["ipc"].get("gen"))  # a view: the engine scatters from the zone

            def on_imported(ev, zone=zone, off=off, handed=handed):
                handed.append(True)
                zone.release_after(off, ev)

            packet = KVPacket(d["request_id"], list(d["prompt_ids"]), int(d["first_token"]), kv,
                              int(d["block_size"]), dict(d.get("sampling") or {}), d.get("ttft_ms"),
                              ready=ready, on_imported=on_imported)
            self.ipc_imports += 1
        else:
            packet = packet_for_import(d, self.engine.device)
        sp = SamplingParams(**packet.sampling) if packet.sampling else SamplingParams()
        if not self.async_engine.running:
            self.async_engine.start()
        try:
            seq = await self.async_engine.submit(packet.request_id, [], sp, user_data={"import_packet": packet})
        except Exception:
            # the engine failed before importing it: free the slot now (a cancelled caller does not free it:
            # the queued import still runs and releases it behind its scatter)
            if packet.on_imported is not None and not handed:
                self._landing_zone().release(off)
            raise
        return {"success": True, "outputs": await self._output(
            seq.output_ids, prompt_len=seq.prompt_len, finish_reason=seq.finish_reason or "length",
            ttft_ms=packet.ttft_ms, latency_ms=seq.latency_ms())}

    async def predict_batch(self, inputs_list: List[Any]) -> List[Dict[str, Any]]:
        return list(await asyncio.gather(*(self.predict(x) for x in inputs_list)))

    async def handle_op(self, op: str, msg: Dict[str, Any]) -> Dict[str, Any]:
        if op == "engine_stats":
            st = self.async_engine.stats()
            if self._decode_link is not None:
                st["kv_link"] = self._decode_link.stats()
            if self._zone is not None:
                z = self._zone
                z._reap()
                st["kv_zone"] = {"slots_used": len(z._used), "reserved": len(z._reserved_at),
                                 "pending_release": len(z._pending), "expired": z.expired,
                                 "capacity": z.capacity}
            return {"success": True, "stats": st}
        if op == "kv_import":
            return await self._kv_import(msg)
        if op == "kv_channel":  # same-node prefill workers map this GPU's landing zone (IPC)
            if self.engine.device.type != "cuda":
                return {"success": False, "error": "no GPU landing zone on a CPU engine"}
            z = self._landing_zone()
            return {"success": True, "handle": z.handle, "handles": z.handles, "seg_bytes": z.seg_bytes,
                    "capacity": z.capacity, "device": str(z.device), "pid": os.getpid()}
        if op == "kv_reserve":  # optionally wait up to wait_s for slots to come back (no host sync: polling)
            zone, n = self._landing_zone(), int(msg["nbytes"])
            if n > zone.seg_bytes:
                return {"success": False, "offset": None, "error": "packet larger than a landing-zone segment"}
            deadline = time.monotonic() + float(msg.get("wait_s") or 0.0)
            off = zone.reserve(n)
            while off is None and time.monotonic() < deadline:
                await asyncio.sleep(0.0005)
                off = zone.reserve(n)
            return {"success": off is not None, "offset": off, "ttl_s": zone.reserve_ttl_s,
                    "gen": zone.generation(off) if off is not None else None}
        if op == "kv_release":  # a sender gave up on a reserved slot (copy or kv_import failed)
            return {"success": self._landing_zone().release(int(msg["offset"]), msg.get("gen"))}
        raise ValueError(f"unsupported op {op}")

    def get_metrics(self) -> Dict[str, Any]:
        m = {
            "model_name": self.config.model_name,
            "request_count": self.request_count,
            "error_count": self.error_count,
            "avg_latency": self.total_latency / self.request_count if self.request_count else 0.0,
            "engine": self.engine.get_stats(),
        }
        if self._decode_link is not None:  # disaggregated prefill: how the prompt KV has travelled
            m["kv_link"] = self._decode_link.stats()
        if self.preproc is not None:  # which processes tokenised / detokenised, in how many calls
            m["preproc"] = self.preproc.stats()
        if self.engine.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.engine.device)
            m["hbm_used_gib"] = (total - free) / 2**30
            m["hbm_total_gib"] = total / 2**30
        return m
