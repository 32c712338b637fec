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
    """bench.py's watchdog around the cross-GPU probe: a stall after the timed region still prints rank 0's
    result line (probe marked as stalled) and ends the process with status 0; a normal emit prints once."""
    import json
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "d = bench._Watchdog({'value': 1.0, 'notes': {}}, 0, 0.5); time.sleep(30)") % root
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and time.time() - t0 < 20, (p.returncode, p.stderr[-2000:])
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and "error" in lines[0]["notes"]["xgpu_probe"], p.stdout
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "d = bench._Watchdog({'value': 2.0, 'notes': {}}, 0, 30); d.emit(); d.emit(); d.cancel()") % root
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1 and lines[0]["value"] == 2.0, p.stdout
