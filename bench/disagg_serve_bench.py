"""Disaggregated serving as TWO worker processes (BASELINE config 3): a prefill worker (role prefill)
ships each prompt's KV into the decode worker's IPC landing zone (kv_reserve → device copy on a
transfer stream → kv_import; the decode engine scatters straight from the zone) and the decode worker
generates. On an 8-GPU node the two sit on different GPUs and the copy rides xGMI; on the one-GPU box
both share the GPU (the protocol and the event-loop behaviour are what is measured, not xGMI).

Closed waves of --batch requests (512 -> 128 tokens) sent to the prefill worker's RPC port, like
bench.py. Reports req/s, p50 / p99 end-to-end latency and TTFT p50 / p99 (measured by the prefill
worker, carried in the reply), plus the decode worker's landing-zone counters. One JSON line."""

import argparse
import asyncio
import json
import os
import random
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from src.client import InferenceClient  # noqa: E402


def spawn(args, role, extra):
    fd, pf = tempfile.mkstemp()
    os.close(fd)
    os.unlink(pf)
    cmd = [sys.executable, "-m", "src.worker", "--worker-id", f"{role}-w", "--host", "127.0.0.1", "--port", "0",
           "--port-file", pf, "--model", "llama", "--arch", "llama", "--preset", args.preset, "--role", role,
           "--max-batch-size", str(args.batch), "--max-model-len", "1024", "--num-kv-blocks", str(args.kv_blocks),
           "--max-latency-ms", "10",
           "--device", args.prefill_device if role == "prefill" else args.decode_device] + extra
    log = open(f"{args.log_dir}/disagg_{role}.log", "w")
    proc = subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT)
    t0 = time.time()
    while not os.path.exists(pf):
        if proc.poll() is not None or time.time() - t0 > 300:
            raise RuntimeError(f"{role} worker failed to start (see {args.log_dir}/disagg_{role}.log)")
        time.sleep(0.2)
    return proc, int(open(pf).read())


async def run(args, pport, dport):
    c = InferenceClient(f"127.0.0.1:{pport}", timeout=600)
    rng = random.Random(3)

    async def one(i, prompt):
        t0 = time.perf_counter()
        r = await c.call({"model": "llama", "inputs": {"prompt_token_ids": prompt, "max_tokens": args.gen_len,
                                                         "ignore_eos": True}})
        assert r["success"], r
        o = r["outputs"]
        assert o["disaggregated"] and o["num_output_tokens"] == args.gen_len, o
        return time.perf_counter() - t0, o.get("ttft_ms")

    def wave():
        return [[rng.randrange(3, 128000) for _ in range(args.prompt_len)] for _ in range(args.batch)]

    for _ in range(args.warmup):
        await asyncio.gather(*(one(i, p) for i, p in enumerate(wave())))
    waves = [wave() for _ in range(args.steps)]
    t0 = time.perf_counter()
    res = []
    for w in waves:
        res += await asyncio.gather(*(one(i, p) for i, p in enumerate(w)))
    el = time.perf_counter() - t0
    lat = sorted(x[0] * 1e3 for x in res)
    ttft = sorted(x[1] for x in res if x[1] is not None)
    st = await InferenceClient(f"127.0.0.1:{dport}").call({"op": "engine_stats", "model": "llama"})
    link = (await c.call({"op": "engine_stats", "model": "llama"}))["stats"].get("kv_link") or {}
    c.close()
    # the point of config 3 is that the KV never crosses the socket: a silent fallback to bytes is a failure
    if link.get("wire_packets", 0) or not link.get("ipc"):
        raise SystemExit(f"disaggregation fell back to the RPC byte path: {link}")
    return {"bench": "disagg_two_process", "preset": args.preset, "req_per_s": round(len(res) / el, 2),
            "p50_latency_ms": round(statistics.median(lat), 1), "p99_latency_ms": round(lat[int(0.99 * len(lat)) - 1], 1),
            "ttft_p50_ms": round(statistics.median(ttft), 1) if ttft else None,
            "ttft_p99_ms": round(ttft[int(0.99 * len(ttft)) - 1], 1) if ttft else None,
            "batch": args.batch, "waves": args.steps, "prompt_len": args.prompt_len, "gen_len": args.gen_len,
            "kv_zone": st.get("stats", {}).get("kv_zone"), "kv_link": link, "kv_path": link.get("kv_path"),
            "devices": {"prefill": args.prefill_device, "decode": args.decode_device}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--kv-blocks", type=int, default=16384)
    ap.add_argument("--log-dir", default="/tmp")
    ap.add_argument("--prefill-device", default="cuda:0")
    ap.add_argument("--decode-device", default="cuda:0", help="cuda:1 on a multi-GPU node: the KV rides xGMI")
    args = ap.parse_args()
    dproc, dport = spawn(args, "decode", [])
    try:
        pproc, pport = spawn(args, "prefill", ["--decode-worker", f"127.0.0.1:{dport}"])
        try:
            print(json.dumps(asyncio.run(run(args, pport, dport))), flush=True)
        finally:
            pproc.terminate()
            pproc.wait(60)
    finally:
        dproc.terminate()
        dproc.wait(60)


if __name__ == "__main__":
    main()
