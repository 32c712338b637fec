"""The example scripts stay runnable (the reference's examples/ are part of the API
surface). Each demo runs as its own process on CPU; the interactive ones get ``exit`` on stdin.

Reference counterparts: examples/batcher_demo.py:23-204, examples/load_balancer_demo.py:27-238,
examples/kvstore_demo.py:19-228, examples/router_demo.py:24-322, examples/worker_demo.py:26-243.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, args=(), stdin=None, timeout=120):
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), *args], input=stdin,
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert p.returncode == 0, f"{script} exited {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    return p.stdout + p.stderr


def test_batcher_demo_scenarios():
    out = _run("batcher_demo.py")
    # the reference's expected flush pattern (batcher_demo.py:30-41, 114-140), both scenarios reached
    assert "batches [5, 5, 2]" in out
    assert "batches [1, 1, 1]" in out


def test_load_balancer_demo_all_strategies():
    out = _run("load_balancer_demo.py", ["--requests", "20"])
    for s in ("round_robin", "least_connections", "random", "least_latency"):
        assert s.upper() in out.upper()


@pytest.mark.parametrize("script", ["kvstore_demo.py", "router_demo.py", "worker_demo.py"])
def test_interactive_demo_exits_cleanly(script):
    _run(script, stdin="help\nexit\n")
