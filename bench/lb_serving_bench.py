#!/usr/bin/env python3
"""
BASELINE config 5's load balancer on real LLM worker processes — the one-GPU rehearsal of the node section's
``lb_serving`` part (src/parallel/node_bench.py):

    closed-loop clients → coordinator (least_latency | round_robin) → K worker processes (src.worker, RPC)

All K workers share one device (``--device``, default cuda:0) and ``--slow`` of them are handicapped with a smaller
decode batch cap (``--slow-batch``), so one replica drains its queue slower than the others — what a busier or
smaller GPU looks like to the balancer. ``least_latency`` scores every request against the workers' engine reports
(piggybacked on replies and health answers: queue, prefill backlog, step time, KV use); ``round_robin`` ignores
them. Every strategy gets its own fresh prefix set of config 5's workload (mixed 128-2048 -> 32-256 tokens, Zipf
shared prefixes, KV pools below the working set so they evict), after a shared warm-up. One JSON line per strategy,
then a summary line with the p50 / p99 ratios.

    python bench/lb_serving_bench.py --preset llama3-8b --workers 3 --slow 1 --requests 192 --concurrency 48

(``--device cpu`` with ``--preset llama-tiny``: the plumbing on CPU, for tests.) Reference:
`/root/reference/src/load_balancer.py:276-291`, `/root/reference/docs/router_vs_load_balancer.md:41-57`.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from src.parallel.lb_serving import LBWorkload, make_requests, serve_through_coordinator  # noqa: E402


def spawn(wid: str, a, batch: int):
    fd, pf = tempfile.mkstemp()
    os.close(fd)
    os.unlink(pf)
    arch = "mixtral" if a.preset.startswith("mixtral") else "llama"
    cmd = [sys.executable, "-m", "src.worker", "--worker-id", wid, "--host", "127.0.0.1", "--port", "0",
           "--port-file", pf, "--model", "llm", "--arch", arch, "--preset", a.preset, "--max-batch-size", str(batch),
           "--max-model-len", str(a.prompt_max + 256 + 16), "--device", a.device, "--num-kv-blocks", str(a.kv_blocks),
           "--kv-block-ttl-s", "30", "--max-latency-ms", "2"]
    if a.device == "cpu":
        cmd.append("--no-graph")
    log = open(os.path.join(tempfile.gettempdir(), f"lbbench-{wid}.log"), "w")
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=log)
    return p, pf, log


def wait_port(p, pf: str, wid: str, timeout: float = 900.0) -> str:
    deadline = time.time() + timeout
    while time.time() < deadline:
        if os.path.exists(pf):
            time.sleep(0.05)
            with open(pf) as f:
                return f"127.0.0.1:{int(f.read().strip())}"
        if p.poll() is not None:
            raise RuntimeError(f"worker {wid} exited with {p.returncode}; see its log under {tempfile.gettempdir()}")
        time.sleep(0.2)
    raise RuntimeError(f"worker {wid} did not start within {timeout:.0f} s")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--slow", type=int, default=1, help="workers with the smaller batch cap")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--slow-batch", type=int, default=8)
    ap.add_argument("--kv-blocks", type=int, default=2048, help="per worker (16 tokens each)")
    ap.add_argument("--requests", type=int, default=192)
    ap.add_argument("--concurrency", type=int, default=48)
    ap.add_argument("--prefixes", type=int, default=24)
    ap.add_argument("--prompt-min", type=int, default=128)
    ap.add_argument("--prompt-max", type=int, default=2048)
    ap.add_argument("--gen", default="32,64,128,256")
    ap.add_argument("--strategies", default="least_latency,round_robin")
    ap.add_argument("--vocab", type=int, default=None)
    a = ap.parse_args(argv)
    if a.vocab is None:
        from src.models.presets import get_preset

        a.vocab = get_preset(a.preset).vocab_size
    gens = tuple(int(x) for x in a.gen.split(","))
    procs = []
    try:
        for i in range(a.workers):
            procs.append((f"w{i}", *spawn(f"w{i}", a, a.slow_batch if i < a.slow else a.batch)))
        workers = {wid: wait_port(p, pf, wid) for wid, p, pf, _ in procs}
        shape = dict(prompt_min=a.prompt_min, prompt_max=a.prompt_max, gen_choices=gens, prefixes=a.prefixes)
        warm = make_requests(LBWorkload(requests=2 * a.workers, seed=999, **shape), a.vocab)
        res = {}
        for i, strat in enumerate(s for s in a.strategies.split(",") if s):
            wl = LBWorkload(requests=a.requests, concurrency=a.concurrency, seed=100 + i, **shape)
            r = asyncio.run(serve_through_coordinator(workers, "llm", "mixtral" if a.preset.startswith("mixtral")
                                                      else "llama", strat, make_requests(wl, a.vocab),
                                                      a.concurrency, warmup=warm))
            r.update(bench="lb_serving_one_device", preset=a.preset, device=a.device, workers=a.workers,
                     slow_workers=a.slow, batch=a.batch, slow_batch=a.slow_batch, kv_blocks_per_worker=a.kv_blocks,
                     concurrency=a.concurrency, data="synthetic token ids, random-init weights")
            res[strat] = r
            print(json.dumps(r), flush=True)
        if "least_latency" in res and "round_robin" in res:
            ll, rr = res["least_latency"], res["round_robin"]
            print(json.dumps({"bench": "lb_serving_one_device_summary",
                              "p99_ll_over_rr": round(ll["p99_latency_ms"] / rr["p99_latency_ms"], 3),
                              "p50_ll_over_rr": round(ll["p50_latency_ms"] / rr["p50_latency_ms"], 3),
                              "req_s_ll_over_rr": round(ll["req_s"] / rr["req_s"], 3),
                              "slow_share_ll": round(sum(ll["per_worker"][f"w{i}"]["dispatched"]
                                                         for i in range(a.slow)) / max(1, ll["requests"]), 3),
                              "slow_share_rr": round(sum(rr["per_worker"][f"w{i}"]["dispatched"]
                                                         for i in range(a.slow)) / max(1, rr["requests"]), 3)}),
                  flush=True)
        return 0
    finally:
        for _, p, _, log in procs:
            p.terminate()
        for _, p, _, log in procs:
            try:
                p.wait(60)
            except subprocess.TimeoutExpired:
                p.kill()
            log.close()


if __name__ == "__main__":
    sys.exit(main())
