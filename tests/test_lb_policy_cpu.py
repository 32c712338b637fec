"""least_latency with an engine-load signal (VERDICT r4 item 5, config 5's balancer) against round-robin and the
size-blind end-to-end-latency EWMA it replaced, on three LLM workers of unequal speed under open-loop arrivals of
mixed prompt / output sizes.

The workers are a discrete-event model of the engine's continuous batching (src/engine/llm_engine.py): a step
is either a prefill of every waiting prompt that fits the batch cap (time = prompt tokens x the worker's prefill
time per token) or one decode step of the running batch (time = the worker's step time, growing a little with the
batch); sequences join and leave the batch between steps. Each worker reports the same ``engine_load`` fields as
:meth:`LLMEngine._update_load_snapshot` — piggybacked on every reply, and on health probes once a second — and
the real :class:`src.load_balancer.LoadBalancer` picks a worker for every arrival. Virtual time: the test is
deterministic and fast."""

import heapq
import random
import statistics

from src.load_balancer import LoadBalancer, LoadBalancerStrategy


class SimWorker:
    def __init__(self, wid, slow, cap=32):
        self.wid, self.slow, self.cap = wid, slow, cap
        self.pf_ms_tok = 0.012 * slow       # 12 us per prompt token at full speed
        self.step_base = 4.0 * slow         # ms per decode step at full speed
        self.waiting, self.running = [], []  # [req]; req = dict(p, g, t0, done)
        self.busy_until = None
        self.step_ema, self.pf_ema = 0.0, 0.0

    def report(self):
        return {"running": len(self.running), "waiting": len(self.waiting),
                "waiting_prompt_tokens": sum(r["p"] for r in self.waiting), "max_num_seqs": self.cap,
                "kv_used_frac": 0.0, "step_ms": self.step_ema, "prefill_us_per_token": self.pf_ema * 1e3}

    def start_step(self, t):
        """Begin the next step at time t; returns its end time (None: idle)."""
        room = self.cap - len(self.running)
        if self.waiting and room > 0:
            batch = self.waiting[:room]
            self.waiting = self.waiting[room:]
            dt = sum(r["p"] for r in batch) * self.pf_ms_tok
            self.pf_ema = self.pf_ms_tok if not self.pf_ema else 0.8 * self.pf_ema + 0.2 * self.pf_ms_tok
            self._pending = ("prefill", batch)
        elif self.running:
            dt = self.step_base * (1.0 + len(self.running) / 64.0)
            self.step_ema = dt if not self.step_ema else 0.8 * self.step_ema + 0.2 * dt
            self._pending = ("decode", None)
        else:
            self.busy_until = None
            return None
        self.busy_until = t + dt
        return self.busy_until

    def end_step(self):
        """Apply the step that just ended; returns the requests it finished."""
        kind, batch = self._pending
        done = []
        if kind == "prefill":
            for r in batch:
                r["done"] = 1
                (done if r["done"] >= r["g"] else self.running).append(r)
        else:
            keep = []
            for r in self.running:
                r["done"] += 1
                (done if r["done"] >= r["g"] else keep).append(r)
            self.running = keep
        return done


def simulate(lb, seed=0, n=1500, rate_per_s=9.0, probe_ms=1000.0):
    rng = random.Random(seed)
    workers = {w.wid: w for w in (SimWorker("fast", 1.0), SimWorker("mid", 1.7), SimWorker("slow", 3.0))}
    for w in workers:
        lb.register_worker(w, f"sim:{w}")
    ev = []  # (time, seq, kind, payload)
    seq = 0
    t = 0.0
    for i in range(n):
        t += rng.expovariate(rate_per_s) * 1e3
        p = rng.choice([32, 64, 128, 512, 512, 1024, 2048])
        g = rng.choice([8, 16, 32, 64, 128, 256, 512])
        heapq.heappush(ev, (t, seq, "arrive", {"p": p, "g": g, "t0": t, "done": 0}))
        seq += 1
    pt = probe_ms
    while pt < t + 120e3:
        heapq.heappush(ev, (pt, seq, "probe", None))
        seq += 1
        pt += probe_ms
    lats = []
    while ev and len(lats) < n:
        now, _, kind, x = heapq.heappop(ev)
        if kind == "arrive":
            wid, _ = lb.pick(cost=(x["p"], x["g"]))
            lb.acquire(wid, (x["p"], x["g"]))
            w = workers[wid]
            w.waiting.append(x)
            if w.busy_until is None:
                end = w.start_step(now)
                heapq.heappush(ev, (end, seq, "step", wid))
                seq += 1
        elif kind == "step":
            w = workers[x]
            for r in w.end_step():
                lat = now - r["t0"]
                lats.append(lat)
                lb.release(x)
                lb.record(x, True, lat / 1e3)
                lb.observe(x, w.report())  # piggybacked on the reply
            end = w.start_step(now)
            if end is not None:
                heapq.heappush(ev, (end, seq, "step", x))
                seq += 1
        else:  # health probe: every worker's report
            for wid, w in workers.items():
                lb.observe(wid, w.report())
    return lats


class E2ELatencyLB(LoadBalancer):
    """The round-4 least_latency: end-to-end latency EWMA x (1 + active requests), blind to request size."""

    def observe(self, worker_id, report):
        pass

    def _least_latency(self, ids, group=None, cost=None):
        cold = [w for w in ids if self.worker_stats[w].ewma_latency is None
                and self.worker_stats[w].active_connections == 0]
        if cold:
            return cold[0]
        return min(ids, key=lambda w: (self.worker_stats[w].ewma_latency or 0.0)
                   * (1.0 + self.worker_stats[w].active_connections))


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def test_engine_load_least_latency_beats_round_robin_and_e2e_latency():
    res = {}
    for name, lb in (("round_robin", LoadBalancer(LoadBalancerStrategy.ROUND_ROBIN)),
                     ("e2e_latency", E2ELatencyLB(LoadBalancerStrategy.LEAST_LATENCY)),
                     ("engine_load", LoadBalancer(LoadBalancerStrategy.LEAST_LATENCY))):
        runs = [simulate(lb.__class__(lb.strategy), seed=s) for s in range(3)]
        lats = [x for r in runs for x in r]
        res[name] = (statistics.median(lats), _pct(lats, 0.99))
    new = res["engine_load"]
    for base in ("round_robin", "e2e_latency"):
        assert new[0] < res[base][0] and new[1] < res[base][1], res


def test_expected_ms_orders_by_backlog_speed_and_size():
    lb = LoadBalancer(LoadBalancerStrategy.LEAST_LATENCY)
    lb.register_worker("a", "x:1")
    lb.register_worker("b", "x:2")
    base = {"running": 4, "waiting": 0, "waiting_prompt_tokens": 0, "max_num_seqs": 32, "kv_used_frac": 0.1,
            "step_ms": 4.0, "prefill_us_per_token": 12.0}
    lb.observe("a", dict(base))
    lb.observe("b", dict(base, step_ms=8.0))  # twice as slow per token
    assert lb.pick(cost=(128, 256))[0] == "a"
    # a long prefill backlog on the fast worker outweighs its speed for a short request
    lb.observe("a", dict(base, waiting=6, waiting_prompt_tokens=60000))
    assert lb.pick(cost=(64, 16))[0] == "b"
    # dispatches since the last report count until the next one arrives
    lb.observe("a", dict(base))
    for _ in range(6):
        lb.acquire("a", (8000, 16))
    assert lb.expected_ms("a", (64, 16)) > lb.expected_ms("b", (64, 16))
    lb.observe("a", dict(base))
    assert lb.worker_stats["a"].unreported_prompt_tokens == 0


def test_reports_cover_only_the_dispatches_they_saw():
    """a reply's engine report covers the dispatches up to the sequence number the worker had received
    (``lb_seen``); later ones (still on the wire) stay counted, so a burst does not herd onto the worker that just
    replied. Reports of another balancer (other token) or without a sequence number cover everything."""
    lb = LoadBalancer(LoadBalancerStrategy.LEAST_LATENCY)
    lb.register_worker("a", "x:1")
    base = {"running": 0, "waiting": 0, "waiting_prompt_tokens": 0, "max_num_seqs": 32, "kv_used_frac": 0.0,
            "step_ms": 4.0, "prefill_us_per_token": 12.0}
    seqs = [lb.acquire("a", (1000, 16)) for _ in range(5)]
    assert seqs == sorted(seqs) and lb.worker_stats["a"].unreported_requests == 5
    lb.observe("a", dict(base, lb=lb.token, lb_seen=seqs[2]))
    assert lb.worker_stats["a"].unreported_requests == 2
    assert lb.worker_stats["a"].unreported_prompt_tokens == 2000
    lb.observe("a", dict(base, lb="other-balancer", lb_seen=seqs[3]))
    assert lb.worker_stats["a"].unreported_requests == 0
    lb.acquire("a", (10, 1))
    lb.observe("a", dict(base))
    assert lb.worker_stats["a"].unreported_requests == 0


def test_health_answer_per_model_reports():
    """a multi-model worker's health answer carries one report per model; a balancer takes its own."""
    lb_a = LoadBalancer(LoadBalancerStrategy.LEAST_LATENCY, model="a")
    lb_b = LoadBalancer(LoadBalancerStrategy.LEAST_LATENCY, model="b")
    reply = {"models": ["a", "b"], "engine_load": {"running": 1},
             "engine_loads": {"a": {"running": 1}, "b": {"running": 7}}}
    assert lb_a.report_of(reply) == {"running": 1} and lb_b.report_of(reply) == {"running": 7}
    old = {"models": ["a", "b"], "engine_load": {"running": 1}}  # a worker without per-model reports
    assert lb_b.report_of(old) is None
    assert lb_a.report_of({"models": ["a"], "engine_load": {"running": 3}}) == {"running": 3}


def test_lb_serving_bench_real_worker_processes_cpu(capsys):
    """bench/lb_serving_bench.py on CPU: three real worker processes (src.worker, RPC) behind the coordinator, one
    with a smaller batch cap; both strategies serve config 5's mixed, prefix-sharing workload completely, every
    request is dispatched to some worker and the summary compares them (the GPU rehearsal is
    tests/test_serving_gpu.py::test_lb_serving_rehearsal_one_gpu)."""
    import importlib.util
    import json
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench", "lb_serving_bench.py")
    spec = importlib.util.spec_from_file_location("lb_serving_bench", path)
    lb_serving_bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lb_serving_bench)

    rc = lb_serving_bench.main(["--preset", "llama-tiny", "--device", "cpu", "--workers", "3", "--slow", "1",
                                "--batch", "8", "--slow-batch", "2", "--kv-blocks", "64", "--requests", "24",
                                "--concurrency", "8", "--prompt-min", "16", "--prompt-max", "64", "--gen", "4,8"])
    assert rc == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.splitlines() if x.startswith("{")]
    runs = {x["strategy"]: x for x in lines if "strategy" in x}
    assert set(runs) == {"least_latency", "round_robin"}
    for r in runs.values():
        assert r["requests"] == 24 and r["error_count"] == 0
        assert sum(p["dispatched"] for p in r["per_worker"].values()) == 24
    assert runs["round_robin"]["per_worker"]["w0"]["dispatched"] == 8  # round robin ignores the slow worker's state
    assert lines[-1]["bench"] == "lb_serving_one_device_summary"


def test_unreported_dispatches_are_bounded_for_silent_workers():
    """A worker that never reports (mock models) must not grow the balancer's unreported-dispatch list without end."""
    from src.load_balancer import UNREPORTED_MAX

    lb = LoadBalancer(LoadBalancerStrategy.ROUND_ROBIN)
    lb.register_worker("m", "x:1")
    for _ in range(UNREPORTED_MAX + 500):
        lb.release("m") if lb.acquire("m", (4, 1)) < 0 else lb.release("m")
    assert lb.worker_stats["m"].unreported_requests == UNREPORTED_MAX
