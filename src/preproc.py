"""
Pre-processing: request normalisation and tokenisation
(promised at `/root/reference/README.md:34,96-98`, absent from the reference).

* :class:`ByteTokenizer` — a deterministic byte-level tokenizer that needs no
  files (no network for HF downloads): ids 0/1/2 are pad/bos/eos, byte ``b``
  is id ``b + 3``. A local HF tokenizer directory can be used instead through
  :func:`load_tokenizer`.
* :func:`normalize_request` — validates an LLM request's ``inputs`` and turns
  it into :class:`GenerationInputs`.
* :class:`PreprocPool` — pushes CPU-bound tokenisation to a separate process
  pool ("disaggregated inference": pre/post-processing out of the worker's
  event loop, `README.md:15,96-98`).
"""

from __future__ import annotations

import asyncio
import concurrent.futures as cf
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

PAD_ID, BOS_ID, EOS_ID = 0, 1, 2
_BYTE_OFFSET = 3


class ByteTokenizer:
    """Byte-level tokenizer. Any id ≥ 259 (a random-init model emits them)
    decodes to a byte by folding it into range, so detokenisation is total."""

    def __init__(self, vocab_size: int = 128256):
        self.vocab_size = vocab_size
        self.pad_token_id, self.bos_token_id, self.eos_token_id = PAD_ID, BOS_ID, EOS_ID

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [b + _BYTE_OFFSET for b in text.encode("utf-8")]
        return ([BOS_ID] + ids) if add_bos else ids

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        out = bytearray()
        for i in ids:
            if i < _BYTE_OFFSET:
                if not skip_special:
                    out += b"<" + str(i).encode() + b">"
                continue
            out.append((i - _BYTE_OFFSET) % 256)
        return out.decode("utf-8", errors="replace")


def load_tokenizer(path: Optional[str] = None, vocab_size: int = 128256):
    """A local HuggingFace tokenizer when ``path`` holds one, else ByteTokenizer."""
    if path:
        try:
            from transformers import AutoTokenizer  # type: ignore

            return AutoTokenizer.from_pretrained(path, local_files_only=True)
        except Exception:
            pass
    return ByteTokenizer(vocab_size)


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 0.0          # 0 → greedy
    top_k: int = 0                    # 0 → disabled
    top_p: float = 1.0
    seed: Optional[int] = None
    ignore_eos: bool = False
    stop_token_ids: List[int] = field(default_factory=list)

    def __post_init__(self):
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not (0.0 < self.top_p <= 1.0):
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k < 0:
            raise ValueError("top_k must be >= 0")

    @property
    def greedy(self) -> bool:
        return self.temperature == 0.0 or self.top_k == 1


@dataclass
class GenerationInputs:
    prompt_token_ids: List[int]
    sampling: SamplingParams
    prompt: Optional[str] = None
    return_text: bool = True


_SAMPLING_KEYS = ("max_tokens", "temperature", "top_k", "top_p", "seed", "ignore_eos", "stop_token_ids")


def normalize_request(inputs: Any, tokenizer=None, max_model_len: Optional[int] = None) -> GenerationInputs:
    """Accepts a prompt string, a token-id list, or a dict with ``prompt`` /
    ``prompt_token_ids`` plus sampling fields."""
    tok = tokenizer or ByteTokenizer()
    if isinstance(inputs, str):
        inputs = {"prompt": inputs}
    elif isinstance(inputs, (list, tuple)) and all(isinstance(x, int) for x in inputs):
        inputs = {"prompt_token_ids": list(inputs)}
    if not isinstance(inputs, dict):
        raise ValueError("LLM inputs must be a prompt string, a token id list, or an object")
    prompt = inputs.get("prompt")
    ids = inputs.get("prompt_token_ids")
    if ids is None:
        if not isinstance(prompt, str):
            raise ValueError("inputs need 'prompt' (str) or 'prompt_token_ids' (list[int])")
        ids = tok.encode(prompt)
    if not ids:
        raise ValueError("empty prompt")
    ids = list(map(int, ids))  # C-speed conversion + range check: ~0.1 us/token on the serving path
    vs = getattr(tok, "vocab_size", None)
    if vs and (min(ids) < 0 or max(ids) >= vs):
        raise ValueError("prompt token id out of vocabulary range")
    sp = SamplingParams(**{k: inputs[k] for k in _SAMPLING_KEYS if k in inputs})
    if max_model_len is not None and len(ids) + sp.max_tokens > max_model_len:
        raise ValueError(f"prompt ({len(ids)}) + max_tokens ({sp.max_tokens}) exceeds max_model_len {max_model_len}")
    return GenerationInputs(prompt_token_ids=ids, sampling=sp, prompt=prompt,
                            return_text=bool(inputs.get("return_text", True)))


_POOL_TOKENIZERS: Dict[Tuple[Optional[str], int], Any] = {}


def _pool_tokenizer(path: Optional[str], vocab_size: int):
    """The tokenizer of a pool process (loaded once per process and kept)."""
    key = (path, vocab_size)
    tok = _POOL_TOKENIZERS.get(key)
    if tok is None:
        tok = _POOL_TOKENIZERS[key] = load_tokenizer(path, vocab_size)
    return tok


def _encode_batch(texts: List[str], vocab_size: int, path: Optional[str] = None) -> Tuple[List[List[int]], int]:
    tok = _pool_tokenizer(path, vocab_size)
    return [list(tok.encode(t)) for t in texts], os.getpid()


def _decode_batch(seqs: List[List[int]], vocab_size: int, path: Optional[str] = None) -> Tuple[List[str], int]:
    tok = _pool_tokenizer(path, vocab_size)
    return [tok.decode(s) for s in seqs], os.getpid()


def _warm(path: Optional[str], vocab_size: int) -> int:
    _pool_tokenizer(path, vocab_size)
    return os.getpid()


class PreprocPool:
    """Tokenise / detokenise in separate processes so that the serving loop never spends its own time on it
    (the reference's "pre/post-processing in a separate process", `/root/reference/README.md:15,96-98`).

    Requests that arrive in the same event-loop turn are coalesced into ONE call to the pool (one pickle round
    trip for a burst of prompts), up to ``max_batch`` texts per call. The processes are started with ``spawn``
    (never ``fork``: the worker process holds a HIP context and an engine thread) and warmed at construction, so
    the first request does not pay the interpreter start-up. ``pids`` records which processes did the work."""

    def __init__(self, processes: int = 2, vocab_size: int = 128256, tokenizer_path: Optional[str] = None,
                 max_batch: int = 64):
        import multiprocessing as mp

        self.vocab_size = vocab_size
        self.path = tokenizer_path
        self.max_batch = max_batch
        self._pool = cf.ProcessPoolExecutor(max_workers=processes, mp_context=mp.get_context("spawn"))
        self.pids: set = set()
        self.calls = 0
        self.items = 0
        self._pending: Dict[str, List[Tuple[Any, asyncio.Future]]] = {"enc": [], "dec": []}
        self._tasks: set = set()  # in-flight pool calls (the loop keeps only weak references to tasks)
        self._scheduled: Dict[str, bool] = {"enc": False, "dec": False}
        # start every process now (and load its tokenizer): a cold spawn costs ~0.1-1 s
        warm = [self._pool.submit(_warm, self.path, vocab_size) for _ in range(processes)]
        for f in warm:
            self.pids.add(f.result(timeout=120))

    async def encode(self, texts: List[str]) -> List[List[int]]:
        loop = asyncio.get_running_loop()
        out, pid = await loop.run_in_executor(self._pool, _encode_batch, list(texts), self.vocab_size, self.path)
        self._account(pid, len(texts))
        return out

    async def decode(self, seqs: List[List[int]]) -> List[str]:
        loop = asyncio.get_running_loop()
        out, pid = await loop.run_in_executor(self._pool, _decode_batch, [list(s) for s in seqs], self.vocab_size,
                                              self.path)
        self._account(pid, len(seqs))
        return out

    def _account(self, pid: int, n: int) -> None:
        self.pids.add(pid)
        self.calls += 1
        self.items += n

    # --- coalesced single-item forms (the serving path)
    def encode_one(self, text: str) -> "asyncio.Future":
        return self._enqueue("enc", text)

    def decode_one(self, ids: List[int]) -> "asyncio.Future":
        return self._enqueue("dec", list(ids))

    def _enqueue(self, kind: str, item: Any) -> "asyncio.Future":
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending[kind].append((item, fut))
        if not self._scheduled[kind]:
            self._scheduled[kind] = True
            loop.call_soon(self._flush, kind)
        return fut

    def _flush(self, kind: str) -> None:
        self._scheduled[kind] = False
        batch, self._pending[kind] = self._pending[kind], []
        for i in range(0, len(batch), self.max_batch):
            t = asyncio.ensure_future(self._run(kind, batch[i:i + self.max_batch]))
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)

    async def _run(self, kind: str, batch: List[Tuple[Any, asyncio.Future]]) -> None:
        items = [x for x, _ in batch]
        try:
            res = await (self.encode(items) if kind == "enc" else self.decode(items))
        except Exception as e:  # noqa: BLE001 — every waiter of the batch gets the failure
            for _, f in batch:
                if not f.done():
                    f.set_exception(e)
            return
        for (_, f), r in zip(batch, res):
            if not f.done():
                f.set_result(r)

    def stats(self) -> Dict[str, Any]:
        return {"processes": sorted(self.pids), "calls": self.calls, "items": self.items}

    def close(self) -> None:
        self._pool.shutdown(wait=False, cancel_futures=True)


def preprocess(inputs: Dict[str, Any]) -> Dict[str, Any]:
    """Generic (non-LLM) normalisation used by the mock path: strip strings,
    lower-case keys."""
    if isinstance(inputs, dict):
        return {str(k).lower(): (v.strip() if isinstance(v, str) else v) for k, v in inputs.items()}
    if isinstance(inputs, str):
        return inputs.strip()  # type: ignore[return-value]
    return inputs


def request_cost(inputs: Any) -> Optional[Tuple[int, int]]:
    """(prompt tokens, max output tokens) of an LLM request as a load balancer can estimate it without the
    worker's tokenizer (text prompts: ~4 bytes per token), or None for other payloads."""
    if not isinstance(inputs, dict):
        return None
    ids = inputs.get("prompt_token_ids")
    if isinstance(ids, list):
        p = len(ids)
    elif isinstance(inputs.get("prompt"), str):
        p = len(inputs["prompt"].encode()) // 4 + 1
    else:
        return None
    try:
        g = int(inputs.get("max_tokens", SamplingParams.max_tokens))
    except (TypeError, ValueError):
        g = SamplingParams.max_tokens
    return p, max(1, g)

