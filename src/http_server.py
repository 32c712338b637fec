"""
HTTP gateway: an OpenAI-style completions API (plus health and Prometheus metrics) in front of the
coordinator's framed-RPC API. It holds no model state — every request becomes one coordinator RPC
(or one streamed RPC), so any number of gateways can front one coordinator.

    python -m src.http_server --coordinator 127.0.0.1:9000 --port 8000

    POST /v1/completions   {"model", "prompt": str | [token ids], "max_tokens", "temperature",
                            "top_p", "top_k", "seed", "stop_token_ids", "ignore_eos", "stream"}
                           stream=true answers with server-sent events ("data: {...}" chunks,
                           then "data: [DONE]"), text and token ids per chunk
    POST /v1/chat/completions  {"model", "messages": [{"role", "content"}], same sampling keys}:
                           the messages rendered in the Llama-3 chat layout (header / end-of-turn
                           markers as text) plus an open assistant turn; answers "chat.completion"
                           objects, or "chat.completion.chunk" deltas when streaming
    GET  /v1/models        the coordinator's registered models
    GET  /health           200 when the coordinator answers its health RPC
    GET  /metrics          Prometheus text format (requests, errors, latency, tokens)
"""

from __future__ import annotations

import argparse
import asyncio
import json
import time
import uuid
from typing import Any, Dict, Optional

from aiohttp import web
from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest
from prometheus_client.exposition import CONTENT_TYPE_LATEST

from src.client import InferenceClient
from src.utils import setup_logging

_SAMPLING = ("max_tokens", "temperature", "top_p", "top_k", "seed", "stop_token_ids", "ignore_eos")
_ROLES = ("system", "user", "assistant", "tool")


def render_chat(messages: Any) -> str:
    """Llama-3 chat layout: one header + body + end-of-turn per message, then an open assistant
    header for the model to continue. (The tokenizer adds the beginning-of-text token.)"""
    if not isinstance(messages, list) or not messages:
        raise ValueError("messages must be a non-empty list")
    out = []
    for m in messages:
        if not isinstance(m, dict) or m.get("role") not in _ROLES or not isinstance(m.get("content"), str):
            raise ValueError("each message needs a role in %s and a string content" % (_ROLES,))
        out.append(f"<|start_header_id|>{m['role']}<|end_header_id|>\n\n{m['content']}<|eot_id|>")
    out.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(out)


class Gateway:
    def __init__(self, coordinator: str, timeout: float = 600.0):
        self.client = InferenceClient(coordinator, timeout=timeout)
        self.reg = CollectorRegistry()
        self.m_req = Counter("die_http_requests", "completion requests", ["model", "stream"], registry=self.reg)
        self.m_err = Counter("die_http_errors", "failed completion requests", ["model"], registry=self.reg)
        self.m_tok = Counter("die_http_output_tokens", "generated tokens", ["model"], registry=self.reg)
        self.m_lat = Histogram("die_http_latency_seconds", "request latency", ["model"], registry=self.reg,
                               buckets=(0.01, 0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10, 30, 60, 120))
        self.m_ttft = Histogram("die_http_ttft_seconds", "time to first token (engine)", ["model"],
                                registry=self.reg, buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2, 5))

    def app(self) -> web.Application:
        a = web.Application()
        a.router.add_post("/v1/completions", self.completions)
        a.router.add_post("/v1/chat/completions", self.chat_completions)
        a.router.add_get("/v1/models", self.models)
        a.router.add_get("/health", self.health)
        a.router.add_get("/metrics", self.metrics)
        a.on_cleanup.append(self._close)
        return a

    async def _close(self, _app) -> None:
        self.client.close()

    @staticmethod
    def _inputs(body: Dict[str, Any]) -> Dict[str, Any]:
        prompt = body.get("prompt")
        if isinstance(prompt, list) and len(prompt) == 1 and isinstance(prompt[0], (str, list)):
            prompt = prompt[0]  # OpenAI allows a batch of one
        if isinstance(prompt, str):
            inp: Dict[str, Any] = {"prompt": prompt}
        elif isinstance(prompt, list) and all(isinstance(x, int) for x in prompt):
            inp = {"prompt_token_ids": prompt}
        else:
            raise ValueError("prompt must be a string or a list of token ids")
        inp.update({k: body[k] for k in _SAMPLING if k in body and body[k] is not None})
        inp.setdefault("max_tokens", 16)
        return inp

    @staticmethod
    def _choice(out: Dict[str, Any], chat: bool = False) -> Dict[str, Any]:
        c = {"index": 0, "token_ids": out.get("token_ids", []), "finish_reason": out.get("finish_reason"),
             "logprobs": None}
        if chat:
            c["message"] = {"role": "assistant", "content": out.get("text", "")}
        else:
            c["text"] = out.get("text", "")
        return c

    async def completions(self, req: web.Request) -> web.StreamResponse:
        return await self._serve(req, chat=False)

    async def chat_completions(self, req: web.Request) -> web.StreamResponse:
        return await self._serve(req, chat=True)

    async def _serve(self, req: web.Request, chat: bool) -> web.StreamResponse:
        t0 = time.perf_counter()
        try:
            body = await req.json()
            model = body["model"]
            if chat:
                body = dict(body, prompt=render_chat(body.get("messages")))
            inputs = self._inputs(body)
        except (ValueError, KeyError, json.JSONDecodeError) as e:
            return web.json_response({"error": {"message": f"bad request: {e}", "type": "invalid_request"}},
                                     status=400)
        stream = bool(body.get("stream"))
        self.m_req.labels(model, str(stream).lower()).inc()
        cid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24]
        created = int(time.time())
        if not stream:
            rep = await self.client.infer(model, inputs, cache=body.get("cache", True))
            return self._finish(model, cid, created, rep, t0, chat)
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream", "Cache-Control": "no-cache"})
        await resp.prepare(req)
        final: Optional[Dict[str, Any]] = None
        first = True
        try:
            async for frame in self.client.infer_stream(model, inputs):
                if frame.get("done") is False:
                    if chat:
                        delta: Dict[str, Any] = {"content": frame.get("delta_text", "")}
                        if first:
                            delta["role"] = "assistant"
                        chunk = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                                 "choices": [{"index": 0, "delta": delta,
                                              "token_ids": frame.get("delta_token_ids", []), "finish_reason": None}]}
                    else:
                        chunk = {"id": cid, "object": "text_completion", "created": created, "model": model,
                                 "choices": [{"index": 0, "text": frame.get("delta_text", ""),
                                              "token_ids": frame.get("delta_token_ids", []),
                                              "finish_reason": None}]}
                    first = False
                    await resp.write(b"data: " + json.dumps(chunk).encode() + b"\n\n")
                else:
                    final = frame
        except (ConnectionError, asyncio.CancelledError):
            raise  # the HTTP client went away: dropping the RPC stream aborts the request upstream
        if final is None or not final.get("success"):
            self.m_err.labels(model).inc()
            err = {"error": {"message": (final or {}).get("error", "stream ended"), "type": "server_error"}}
            await resp.write(b"data: " + json.dumps(err).encode() + b"\n\n")
        else:
            out = final["outputs"]
            self._observe(model, out, t0)
            end = {"index": 0, "token_ids": [], "finish_reason": out.get("finish_reason")}
            end.update({"delta": {}} if chat else {"text": ""})
            last = {"id": cid, "object": "chat.completion.chunk" if chat else "text_completion", "created": created,
                    "model": model, "choices": [end], "usage": self._usage(out)}
            await resp.write(b"data: " + json.dumps(last).encode() + b"\n\n")
        await resp.write(b"data: [DONE]\n\n")
        await resp.write_eof()
        return resp

    def _observe(self, model: str, out: Dict[str, Any], t0: float) -> None:
        self.m_lat.labels(model).observe(time.perf_counter() - t0)
        self.m_tok.labels(model).inc(out.get("num_output_tokens", 0))
        if out.get("ttft_ms") is not None:
            self.m_ttft.labels(model).observe(out["ttft_ms"] / 1e3)

    @staticmethod
    def _usage(out: Dict[str, Any]) -> Dict[str, int]:
        p, c = int(out.get("num_prompt_tokens", 0)), int(out.get("num_output_tokens", 0))
        return {"prompt_tokens": p, "completion_tokens": c, "total_tokens": p + c}

    def _finish(self, model: str, cid: str, created: int, rep: Dict[str, Any], t0: float,
                chat: bool = False) -> web.Response:
        if not rep.get("success"):
            self.m_err.labels(model).inc()
            status = 404 if "not registered" in str(rep.get("error", "")) else 502
            return web.json_response({"error": {"message": rep.get("error"), "type": "server_error"}}, status=status)
        out = rep["outputs"]
        if not isinstance(out, dict) or "token_ids" not in out:  # a mock model: pass its outputs through
            return web.json_response({"id": cid, "object": "text_completion", "created": created, "model": model,
                                      "outputs": out})
        self._observe(model, out, t0)
        return web.json_response({"id": cid, "object": "chat.completion" if chat else "text_completion",
                                  "created": created, "model": model, "choices": [self._choice(out, chat)],
                                  "usage": self._usage(out), "cached": bool(rep.get("cached"))})

    async def models(self, _req: web.Request) -> web.Response:
        rep = await self.client.call({"op": "models"})
        data = [{"id": m, "object": "model", "versions": v} for m, v in rep.get("models", {}).items()]
        return web.json_response({"object": "list", "data": data})

    async def health(self, _req: web.Request) -> web.Response:
        try:
            rep = await asyncio.wait_for(self.client.call({"op": "health"}), 5.0)
            ok = bool(rep.get("success"))
        except Exception:  # noqa: BLE001 - any failure means unhealthy
            ok = False
        return web.json_response({"healthy": ok}, status=200 if ok else 503)

    async def metrics(self, _req: web.Request) -> web.Response:
        return web.Response(body=generate_latest(self.reg), headers={"Content-Type": CONTENT_TYPE_LATEST})


def main(argv=None) -> None:
    setup_logging()
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--coordinator", default="127.0.0.1:9000")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    a = p.parse_args(argv)
    web.run_app(Gateway(a.coordinator).app(), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
