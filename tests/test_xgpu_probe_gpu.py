"""The cross-GPU probe a multi-GPU bench.py runs after its timed region (src/parallel/xgpu_probe.py), rehearsed
with 2 ranks on this one GPU (gloo coordinates; RCCL refuses two ranks on one device): the one-shot IPC
all-reduce runs without raising its error word, the landing-zone KV hop delivers every byte and a TP=2
engine across the two ranks serves tokens that agree with a TP=1 recompute."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_xgpu_probe_two_ranks_one_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import socket

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), "-m", "src.parallel.xgpu_probe", "--same-device"]
    p = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith('{"bench": "xgpu_probe"')]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(line[0])
    assert r["ipc_allreduce"]["error_word"] is False, r
    assert r["ipc_allreduce"]["32x8192"]["us"] > 0, r
    hop = r["kv_hop"]
    assert hop["per_rank"][1]["receiver_bytes_match"] is True, hop
    assert hop["GBps"] > 0 and all(x["error"] is None for x in hop["per_rank"]), hop
    tpe = r["tp_engine"]  # TP=2 llama-mini over both ranks: graph windows, fused exchange, tokens vs TP=1
    assert tpe.get("graphs_replayed") and tpe.get("fused_exchange") and tpe.get("one_shot_error") is False, tpe
    assert all(tpe["tokens_agree_with_tp1"]), tpe
