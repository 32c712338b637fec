"""HTTP gateway (src/http_server.py) on CPU: OpenAI-style /v1/completions in front of a coordinator
and a tiny-Llama worker — plain and server-sent-event streaming responses agree token for token
with the RPC API, /v1/models lists the registered model, /health and /metrics answer."""

import asyncio
import json

import aiohttp
from aiohttp import web

from src.client import InferenceClient
from src.config import ModelConfig
from src.coordinator import Coordinator
from src.http_server import Gateway, render_chat
from src.worker import Worker


def llm_cfg():
    return ModelConfig(model_name="tiny", model_path="", arch="llama", preset="llama-tiny", max_batch_size=4,
                       max_model_len=256, max_num_batched_tokens=128, num_kv_blocks=128, use_cuda_graph=False,
                       max_latency_ms=1.0, overrides={"device": "cpu"})


def test_openai_completions_plain_and_stream():
    async def main():
        w = Worker("h0", host="127.0.0.1", install_signal_handlers=False)
        assert w.load_model(llm_cfg())
        wport = await w.start()
        coord = Coordinator(port=0, max_batch_size=4, max_latency_ms=2)
        cport = await coord.start()
        await coord.add_static_worker(f"127.0.0.1:{wport}")
        gw = Gateway(f"127.0.0.1:{cport}")
        runner = web.AppRunner(gw.app())
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        base = f"http://127.0.0.1:{port}"
        body = {"model": "tiny", "prompt": "hello world", "max_tokens": 9, "ignore_eos": True}
        rpc = await InferenceClient(f"127.0.0.1:{cport}").infer("tiny", {k: v for k, v in body.items() if k != "model"},
                                                               cache=False)
        async with aiohttp.ClientSession() as s:
            async with s.post(base + "/v1/completions", json=body) as r:
                assert r.status == 200
                plain = await r.json()
            ch = plain["choices"][0]
            assert ch["token_ids"] == rpc["outputs"]["token_ids"] and ch["finish_reason"] == "length"
            assert plain["usage"]["completion_tokens"] == 9 and ch["text"] == rpc["outputs"]["text"]
            toks, text, events = [], "", []
            async with s.post(base + "/v1/completions", json=dict(body, stream=True)) as r:
                assert r.status == 200 and r.headers["Content-Type"].startswith("text/event-stream")
                async for line in r.content:
                    line = line.decode().strip()
                    if not line.startswith("data: "):
                        continue
                    events.append(line[6:])
                    if line[6:] == "[DONE]":
                        break
                    chunk = json.loads(line[6:])
                    toks += chunk["choices"][0]["token_ids"]
                    text += chunk["choices"][0]["text"]
            assert events[-1] == "[DONE]"
            assert toks == ch["token_ids"] and text == ch["text"]
            assert json.loads(events[-2])["choices"][0]["finish_reason"] == "length"
            async with s.get(base + "/v1/models") as r:
                assert [m["id"] for m in (await r.json())["data"]] == ["tiny"]
            async with s.get(base + "/health") as r:
                assert r.status == 200
            async with s.get(base + "/metrics") as r:
                m = await r.text()
                assert 'die_http_requests_total{model="tiny",stream="true"} 1.0' in m
                assert "die_http_output_tokens_total" in m
            # chat: the rendered conversation is an ordinary prompt; plain and streamed agree with RPC
            msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hello"}]
            chat = {"model": "tiny", "messages": msgs, "max_tokens": 7, "ignore_eos": True}
            want = await InferenceClient(f"127.0.0.1:{cport}").infer(
                "tiny", {"prompt": render_chat(msgs), "max_tokens": 7, "ignore_eos": True}, cache=False)
            async with s.post(base + "/v1/chat/completions", json=chat) as r:
                assert r.status == 200
                cj = await r.json()
            assert cj["object"] == "chat.completion" and cj["id"].startswith("chatcmpl-")
            msg = cj["choices"][0]["message"]
            assert msg["role"] == "assistant" and msg["content"] == want["outputs"]["text"]
            assert cj["choices"][0]["token_ids"] == want["outputs"]["token_ids"]
            deltas, roles = [], []
            async with s.post(base + "/v1/chat/completions", json=dict(chat, stream=True)) as r:
                async for line in r.content:
                    line = line.decode().strip()
                    if not line.startswith("data: ") or line[6:] == "[DONE]":
                        continue
                    ch = json.loads(line[6:])
                    assert ch["object"] == "chat.completion.chunk"
                    d = ch["choices"][0]["delta"]
                    roles.append(d.get("role"))
                    deltas += ch["choices"][0]["token_ids"]
            assert roles[0] == "assistant" and deltas == want["outputs"]["token_ids"]
            async with s.post(base + "/v1/chat/completions", json={"model": "tiny", "messages": []}) as r:
                assert r.status == 400
            async with s.post(base + "/v1/completions", json={"model": "nope", "prompt": "x"}) as r:
                assert r.status == 404
            async with s.post(base + "/v1/completions", json={"model": "tiny", "prompt": {"bad": 1}}) as r:
                assert r.status == 400
        await runner.cleanup()
        await coord.stop()
        await w.shutdown()
    asyncio.run(main())
