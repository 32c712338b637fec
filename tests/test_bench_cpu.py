"""bench.py contract on CPU (gloo): the driver launches it under torch.distributed.run with one rank
per GPU and parses ONE JSON line from rank 0. The multi-rank plumbing (process group, barriers
around the timed region, MAX over ranks, latency gather) is exercised here with the reference-op
engine and a tiny preset; the numbers themselves mean nothing on CPU."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--preset", "llama-tiny", "--batch", "4", "--prompt-len", "16", "--gen-len", "4",
         "--max-model-len", "64", "--steps", "2", "--warmup", "1"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc: int, extra):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    if nproc == 1:
        cmd = [sys.executable, "bench.py"] + SMALL + extra
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(nproc)]
        cmd += SMALL + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only, one line
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc,extra,par,replicas", [
    (1, [], "dp1", 1),
    (2, [], "dp2", 2),
    (2, ["--tp", "2"], "dp1-tp2", 1),
])
def test_bench_json_contract(nproc, extra, par, replicas):
    res = _run(nproc, extra)
    assert KEYS <= set(res)
    assert res["n_gpus"] == nproc and res["steps"] == 2 and res["warmup"] == 1
    assert res["unit"] == "req/s" and res["higher_is_better"] is True and res["scaling"] == "weak"
    assert res["config"]["parallelism"] == par
    assert res["config"]["global_batch"] == 4 * replicas
    # value is the whole-job request rate: steps x batch x replicas over the (max-over-ranks) time
    assert res["value"] == pytest.approx(2 * 4 * replicas / (res["ms_per_step"] * 2 / 1e3), rel=0.02)
    assert res["p50_latency_ms"] > 0


def test_bench_watchdog_prints_the_line_once_and_ends_a_stalled_rank():
    """bench.py's watchdog around the post-timed-region node section: a stall still prints rank 0's result line
    once, says so at the top level (``cross_gpu_status``) and in the section (``status`` 3, the stalled part),
    and ends the process with a NON-zero status (a stall must never look like a successful run); a
    normal emit prints once."""
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "d = bench._Watchdog({'value': 1.0, 'notes': {}}, 0, 0.5, {'part': 'tp_wave', 'done': {'disagg': {'req_s_total': 1}}}); "
            "time.sleep(30)") % root
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3 and time.time() - t0 < 20, (p.returncode, p.stderr[-2000:])
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = lines[0]
    assert res["cross_gpu_status"].startswith("stalled in tp_wave")
    assert res["notes"]["cross_gpu"]["status"] == 3 and res["notes"]["cross_gpu"]["stalled_part"] == "tp_wave"
    assert res["notes"]["cross_gpu"]["disagg"] == {"req_s_total": 1}
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "d = bench._Watchdog({'value': 2.0, 'notes': {}}, 0, 30); d.emit(); d.emit(); d.cancel()") % root
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1 and lines[0]["value"] == 2.0, p.stdout


def _self_launched(n: int, extra):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", str(n)] + SMALL + extra
    return subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          timeout=600)


def test_bench_gpus_n_without_launcher_runs_n_real_ranks():
    """``bench.py --gpus 4`` outside torch.distributed.run used to run ONE replica and report
    four. It now starts the launcher as a child: four processes really serve, each reports its identity, and the
    value is four replicas' requests over the slowest replica's time."""
    r = _self_launched(4, ["--cross-gpu", "off"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    n = res["notes"]
    assert res["n_gpus"] == 4 and n["world_size_seen"] == 4 and n["distinct_devices"] == 4
    assert len({d["pid"] for d in n["devices"]}) == 4 and len(n["rank_elapsed_s"]) == 4
    assert res["config"]["parallelism"] == "dp4" and res["config"]["global_batch"] == 16
    assert res["value"] == pytest.approx(2 * 4 * 4 / (res["ms_per_step"] * 2 / 1e3), rel=0.02)


def test_bench_gpus_mismatch_under_launcher_refuses():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4"] + SMALL, cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 2 and not [ln for ln in r.stdout.splitlines() if ln.startswith("{")], r.stdout


def test_bench_node_section_configs_3_4_5_on_cpu():
    """The post-timed-region node section over 2 CPU ranks (gloo): config 3 (prefill worker on rank 0 -> decode
    worker on rank 1 over the RPC; on a CPU engine the KV rides the socket: kv_path 'wire'), config 5 (a worker per
    rank behind one coordinator on rank 0: least_latency then round_robin, mixed lengths with shared prefixes,
    small KV pools that evict) and config 4 (a TP=2 engine over both ranks) all serve; their status reaches the top
    level."""
    r = _self_launched(2, ["--cross-gpu", "on", "--tp-wave-min-world", "2", "--tp-wave-preset", "llama-tiny",
                           "--lb-preset", "mixtral-tiny", "--lb-kv-blocks", "64", "--lb-requests-per-worker", "6"])
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["cross_gpu_status"] == "ok", res["notes"].get("cross_gpu")
    cross = res["notes"]["cross_gpu"]
    assert cross["status"] == 0
    d = cross["disagg"]
    assert d["pairs"] == 1 and d["req_s_total"] > 0 and d["kv_path"] == "wire" and d["ttft_p50_ms"] > 0
    t = cross["tp_wave"]
    assert t["tp"] == 2 and t["requests"] == 4 and t["all_tokens"] and t["req_s"] > 0
    lb = cross["lb_serving"]
    assert lb["workers"] == 2 and [x["strategy"] for x in lb["runs"]] == ["least_latency", "round_robin"], lb
    for run in lb["runs"]:
        assert run["requests"] == 12 and run["error_count"] == 0 and run["req_s"] > 0, run
        assert sum(p["dispatched"] for p in run["per_worker"].values()) == 12, run
    assert lb["prefix_hit_rate"] is not None and lb["p99_latency_ms"] >= lb["p50_latency_ms"] > 0, lb
    assert lb["lru_evictions"] >= 0 and lb["ttl_evictions"] >= 0 and lb["dispatched_per_worker"], lb


def test_bench_node_section_child_run_failure_and_stall():
    """The node section runs in its own launcher (rank 0's child): a run that dies is reported as an error
    (status 1, the exit code), a run past the budget is killed with its process group and reported as a stall
    (status 3) — in both cases rank 0 still has the timed result to print."""
    sys.path.insert(0, ROOT)
    import bench

    state = {"part": None, "done": {}}
    args = bench.parse(SMALL + ["--cross-gpu", "on", "--cross-gpu-budget-s", "1"])
    cross, stalled = bench.run_node_child(args, SMALL + ["--cross-gpu", "on"], 1, state)
    assert stalled and cross["status"] == 3 and "stalled_part" in cross
    args = bench.parse(SMALL + ["--cross-gpu-budget-s", "200"])
    cross, stalled = bench.run_node_child(args, SMALL + ["--batch", "not-a-number"], 1, state)
    assert not stalled and cross["status"] == 1 and "exited" in cross["error"], cross
