"""
Continuous-batching scheduler (iteration-level): the reference Batcher's
max-batch / max-latency flush (`/root/reference/src/batcher.py:144-166`)
re-cast for token generation.

Every engine step is one of

* a **prefill step** — new prompts (and chunks of long prompts: chunked
  prefill) packed into one ragged batch of at most ``max_num_batched_tokens``
  tokens — when nothing is decoding;
* a **decode step** — one token for every running sequence (≤ ``max_num_seqs``),
  replayed from a captured hipGraph;
* a **mixed step** (``EngineConfig.mixed_batching``) — the decode rows of every
  running sequence plus prompt chunks filling the step up to
  ``mixed_step_tokens`` rows, run as ONE ragged batch (a decode row is a 1-token
  chunk). At <= 128 rows every projection is a weight stream on the decode GEMM,
  so the prompt tokens ride along almost for free and running sequences never
  stall behind a whole prefill: per-iteration admission, the continuous form of
  the reference Batcher's size-or-latency flush.

Sequences join the running batch as soon as their prompt is done and leave it
the step they finish, so the batch never waits for its slowest member.
``max_latency_ms`` bounds how long an idle engine waits to accumulate a fuller
first prefill batch. When the KV pool runs dry during decode the most recently
admitted sequence is preempted. Two preemption modes (``EngineConfig.preemption_mode``):

* **recompute** — blocks freed, the sequence re-prefills later (prompt + the
  tokens generated so far); its cached prefix blocks usually make that cheap;
* **swap** — its blocks are packed (``move_blocks`` HIP kernel) and copied to
  pinned host memory; on resume fresh blocks are allocated and the KV is
  scattered back, so nothing is recomputed. ``auto`` swaps long contexts
  (≥ ``swap_min_tokens``) and recomputes short ones.

Swapped sequences resume (FIFO) before any new prompt is admitted.
"""

from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, List, Optional, Tuple

from src.config import EngineConfig
from src.engine.block_manager import KVBlockManager
from src.engine.sequence import Sequence, SeqStatus


@dataclass
class PrefillChunk:
    seq: Sequence
    start: int        # first position computed in this step
    length: int       # tokens computed in this step
    decode: bool = False  # a decode row of a mixed step (1 token: the last sampled one)

    @property
    def completes_prompt(self) -> bool:
        return self.start + self.length >= self.seq.prompt_len

    def tokens(self) -> List[int]:
        s = self.seq
        if self.decode:
            return [s.last_token]
        return s.prompt_ids[self.start: self.start + self.length] if self.start + self.length <= s.prompt_len \
            else [s.token_at(i) for i in range(self.start, self.start + self.length)]


@dataclass
class SchedulerOutput:
    prefill: List[PrefillChunk] = field(default_factory=list)
    decode: List[Sequence] = field(default_factory=list)
    preempted: List[Sequence] = field(default_factory=list)
    # (sequence, block ids) to copy out to host / back in from host before this step's forward
    swap_out: List[Tuple[Sequence, List[int]]] = field(default_factory=list)
    swap_in: List[Tuple[Sequence, List[int]]] = field(default_factory=list)

    @property
    def empty(self) -> bool:
        return not self.prefill and not self.decode

    @property
    def mixed(self) -> bool:
        return bool(self.prefill and self.decode)

    def chunks(self) -> List[PrefillChunk]:
        """A mixed step as one ragged batch: decode rows first (1-token chunks), then prompt chunks."""
        return [PrefillChunk(s, len(s) - 1, 1, decode=True) for s in self.decode] + self.prefill

    @property
    def num_tokens(self) -> int:
        return sum(c.length for c in self.prefill) + len(self.decode)


class Scheduler:
    def __init__(self, cfg: EngineConfig, blocks: KVBlockManager, max_model_len: int,
                 swap_capacity_blocks: int = 0):
        self.cfg = cfg
        self.blocks = blocks
        self.max_model_len = max_model_len
        self.waiting: Deque[Sequence] = deque()
        self.running: List[Sequence] = []
        self.swapped: Deque[Sequence] = deque()
        self.swap_capacity = swap_capacity_blocks   # host swap space, in KV blocks
        self.swap_used = 0
        self.num_swaps_out = 0
        self.num_swaps_in = 0
        self.num_preemptions = 0
        self.steps_prefill = 0
        self.steps_decode = 0
        self.steps_mixed = 0
        self._stalled = False  # the last step was a prefill step that decode-ready sequences waited for
        # while new prompts are held for a larger prefill step (cfg.prefill_batch_tokens): the time by
        # which the oldest must be admitted (the engine sizes its decode windows to end by then)
        self.defer_deadline: Optional[float] = None

    def add(self, seq: Sequence) -> None:
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self.swapped)

    def abort(self, request_id: str) -> Optional[Sequence]:
        for q in (self.waiting, self.running, self.swapped):
            for s in list(q):
                if s.request_id == request_id:
                    q.remove(s)
                    self.blocks.free(s)
                    self._drop_swap(s)
                    s.status = SeqStatus.FINISHED
                    s.finish_reason = "abort"
                    return s
        return None

    # ------------------------------------------------------------- policy
    def _hold_for_batching(self, now: float) -> bool:
        """Idle engine + a partial first batch younger than max_latency: wait."""
        if self.running or not self.waiting:
            return False
        if len(self.waiting) >= self.cfg.max_num_seqs:
            return False
        tokens = sum(s.prompt_len for s in self.waiting)
        if tokens >= self.cfg.max_num_batched_tokens:
            return False
        oldest = self.waiting[0].arrival
        return (now - oldest) * 1e3 < self.cfg.max_latency_ms

    def next_wakeup(self) -> Optional[float]:
        """Seconds until a held batch must be released (for the engine loop)."""
        if not self.waiting or self.running:
            return None
        return max(0.0, self.cfg.max_latency_ms / 1e3 - (time.perf_counter() - self.waiting[0].arrival))

    def schedule(self, now: Optional[float] = None) -> SchedulerOutput:
        now = time.perf_counter() if now is None else now
        out = SchedulerOutput()
        self.defer_deadline = None  # set again below only if this step holds new prompts back
        budget = self.cfg.max_num_batched_tokens
        self._resumed_now = set()
        # 0) resume swapped-out sequences first (FIFO); while one is still parked, admit nothing new
        while self.swapped and len(self.running) < self.cfg.max_num_seqs:
            seq = self.swapped[0]
            nb = self.blocks.blocks_needed(seq.num_computed)
            if nb + len(self.running) // 4 > self.blocks.num_available():
                break
            self.swapped.popleft()
            ids = self.blocks.allocate_fresh(seq, nb)
            out.swap_in.append((seq, ids))
            self.swap_used -= nb
            self.num_swaps_in += 1
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
            self._resumed_now.add(id(seq))
        blocked = bool(self.swapped)
        ready = [s for s in self.running if not s.in_prefill and s.num_computed == len(s) - 1]
        mode = self._mixed_mode()
        mixed = False
        if ready and mode != "off":
            room = min(budget, self.cfg.mixed_step_tokens) - len(ready)
            pending = self._pending_prompt_tokens(blocked)
            # "auto": ride along when the prompt work fits the spare rows; otherwise alternate one bounded
            # prefill step (the decode rows wait for it) with one decode-only step, so decode progresses at
            # least every other step and no prompt is split into ride-along fragments
            # "always" mixes while prompt chunks still get a real share of the step; once the decode rows
            # leave fewer than a quarter of mixed_step_tokens spare it falls back to the alternation below,
            # so running prompts and new arrivals cannot be starved by a large decode batch
            mixed = (mode == "always" and room >= max(1, self.cfg.mixed_step_tokens // 4)) or pending <= room
            if not mixed and self._defer_prefill(now, blocked):
                out.decode = self._schedule_decode(ready, out)
                if out.decode:
                    self.steps_decode += 1
                return out
            if not mixed and self._stalled:
                self._stalled = False
                out.decode = self._schedule_decode(ready, out)
                if out.decode:
                    self.steps_decode += 1
                return out
            if not mixed and pending:
                budget = min(budget, self.cfg.prefill_tokens_while_decoding)
        elif ready and self._defer_prefill(now, blocked):
            out.decode = self._schedule_decode(ready, out)
            if out.decode:
                self.steps_decode += 1
            return out
        self._stalled = False
        if mixed:
            # decode rows first (they are latency-critical); prompt chunks fill the step up to
            # mixed_step_tokens rows
            out.decode = self._schedule_decode(ready, out)
            budget = max(0, min(budget, self.cfg.mixed_step_tokens) - len(out.decode))
        # 1) continue chunked prefills already running
        for seq in self.running:
            if budget <= 0:
                break
            if seq.in_prefill:
                n = min(seq.prompt_len - seq.num_computed, budget)
                out.prefill.append(PrefillChunk(seq, seq.num_computed, n))
                budget -= n
        # 2) admit new prompts
        if not blocked and not self._hold_for_batching(now):
            while self.waiting and budget > 0 and len(self.running) < self.cfg.max_num_seqs:
                seq = self.waiting[0]
                if len(seq) > self.max_model_len:
                    self.waiting.popleft()
                    seq.status = SeqStatus.FINISHED
                    seq.finish_reason = "length_exceeds_max_model_len"
                    out.preempted.append(seq)  # reported back as failed
                    continue
                # reserve one block of headroom per running sequence for decode growth
                if not self.blocks.can_allocate(seq, reserve=len(self.running) // 4):
                    break
                self.waiting.popleft()
                self.blocks.allocate(seq)
                seq.status = SeqStatus.RUNNING
                self.running.append(seq)
                remaining = len(seq) - seq.num_computed
                if seq.imported_kv:
                    continue  # KV shipped from a prefill worker: goes straight to decode
                n = min(seq.prompt_len - seq.num_computed, budget) if seq.in_prefill else remaining
                out.prefill.append(PrefillChunk(seq, seq.num_computed, n))
                budget -= n
        if mixed:
            if out.prefill and out.decode:
                self.steps_mixed += 1
            elif out.prefill:
                self.steps_prefill += 1
            elif out.decode:
                self.steps_decode += 1
            return out
        if out.prefill:
            self.steps_prefill += 1
            self._stalled = bool(ready)  # decode rows waited for this step: the next one decodes
            return out
        # 3) decode everything that is past its prompt
        out.decode = self._schedule_decode(ready, out)
        if out.decode:
            self.steps_decode += 1
        return out

    def _defer_prefill(self, now: float, blocked: bool) -> bool:
        """Hold newly arrived prompts while sequences decode (cfg.prefill_batch_tokens): True while
        fewer than that many prompt tokens wait and the oldest is younger than prefill_batch_wait_ms.
        Chunked prefills already running are never held."""
        self.defer_deadline = None
        want = int(getattr(self.cfg, "prefill_batch_tokens", 0) or 0)
        if want <= 0 or blocked or not self.waiting or any(s.in_prefill for s in self.running):
            return False
        if sum(max(1, len(s) - s.num_computed) for s in self.waiting) >= want:
            return False
        deadline = self.waiting[0].arrival + float(self.cfg.prefill_batch_wait_ms) / 1e3
        if now >= deadline:
            return False
        self.defer_deadline = deadline
        return True

    def _mixed_mode(self) -> str:
        m = self.cfg.mixed_batching
        if m is True:
            return "always"
        if m is False or m is None:
            return "off"
        return str(m)

    def _pending_prompt_tokens(self, blocked: bool) -> int:
        """Prompt tokens that could be scheduled now: unfinished chunked prefills, plus (unless
        admission is blocked) waiting prompts."""
        n = sum(s.prompt_len - s.num_computed for s in self.running if s.in_prefill)
        if not blocked:
            n += sum(max(1, len(s) - s.num_computed) for s in self.waiting)
        return n

    def _schedule_decode(self, ready: List[Sequence], out: SchedulerOutput) -> List[Sequence]:
        """One KV slot for every ready sequence (oldest first), preempting the newest when the pool is dry."""
        ready = sorted(ready, key=lambda s: s.arrival)
        decode: List[Sequence] = []
        for seq in ready:
            if seq.status != SeqStatus.RUNNING:
                continue
            while not self.blocks.ensure_slots(seq, len(seq)):
                victim = self._pick_victim(exclude=seq)
                if victim is None:
                    break
                self._preempt(victim, out)
                out.preempted.append(victim)
                if victim in decode:
                    decode.remove(victim)
            else:
                decode.append(seq)
                continue
            # could not find room even after preempting everyone else
            self._preempt(seq, out)
            out.preempted.append(seq)
        return decode

    def _pick_victim(self, exclude: Sequence) -> Optional[Sequence]:
        """Newest arrival first, but a sequence swapped back in during THIS step goes last: its KV
        is only scattered into its fresh blocks by this step's swap-in, so swapping it straight
        out again would gather uninitialised blocks (scheduler/_run_swaps)."""
        cands = [s for s in self.running if s is not exclude and s.status == SeqStatus.RUNNING]
        if not cands:
            return None
        resumed = getattr(self, "_resumed_now", set())
        return max(cands, key=lambda s: (id(s) not in resumed, s.arrival))

    def _swap_ok(self, seq: Sequence) -> bool:
        mode = self.cfg.preemption_mode
        if self.swap_capacity <= 0 or mode == "recompute" or seq.in_prefill or seq.num_computed == 0:
            return False
        if mode == "auto" and seq.num_computed < self.cfg.swap_min_tokens:
            return False
        return self.swap_used + self.blocks.blocks_needed(seq.num_computed) <= self.swap_capacity

    def _drop_swap(self, seq: Sequence) -> None:
        if seq.status == SeqStatus.SWAPPED:
            self.swap_used -= self.blocks.blocks_needed(seq.num_computed)
            seq.swap_buf = None

    def _preempt(self, seq: Sequence, out: Optional[SchedulerOutput] = None) -> None:
        """Preempt ``seq``: swap its KV to host (see module doc) or drop it for recompute."""
        if seq in self.running:
            self.running.remove(seq)
        self.num_preemptions += 1
        seq.num_preemptions += 1
        if out is not None and self._swap_ok(seq):
            nb = self.blocks.blocks_needed(seq.num_computed)
            out.swap_out.append((seq, list(seq.block_table[:nb])))
            # freed now; the engine gathers them before this step's forward can overwrite any
            self.blocks.free(seq)
            self.swap_used += nb
            self.num_swaps_out += 1
            seq.status = SeqStatus.SWAPPED
            self.swapped.append(seq)
            return
        self.blocks.free(seq)
        seq.num_computed = 0
        seq.imported_kv = False  # the recompute re-prefills locally (prefix matching applies again)
        seq.status = SeqStatus.WAITING
        # the generated tokens become part of the prompt for the recompute
        seq.prompt_ids = seq.prompt_ids + seq.output_ids
        seq.sampling.max_tokens -= len(seq.output_ids)
        seq._preempted_outputs = getattr(seq, "_preempted_outputs", []) + seq.output_ids  # type: ignore[attr-defined]
        seq.output_ids = []
        seq.block_hashes = None
        self.waiting.appendleft(seq)

    # ------------------------------------------------------------ results
    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        seq.finish_time = time.perf_counter()
        if seq in self.running:
            self.running.remove(seq)
        self.blocks.free(seq)

    def stats(self) -> dict:
        return {
            "waiting": len(self.waiting),
            "running": len(self.running),
            "swapped": len(self.swapped),
            "preemptions": self.num_preemptions,
            "swaps_out": self.num_swaps_out,
            "swaps_in": self.num_swaps_in,
            "steps_prefill": self.steps_prefill,
            "steps_decode": self.steps_decode,
            "steps_mixed": self.steps_mixed,
        }
