"""bench.py's multi-GPU path rehearsed on ONE GPU: two ranks share cuda:0 (gloo coordinates; RCCL refuses two
ranks on one device), each serves its data-parallel replica, then the post-timed-region node section runs every
part a real node runs — the cross-GPU transports (xgpu_probe), config 3 (prefill worker on rank 0 -> decode worker
on rank 1, the prompt KV gathered straight into the decode process's IPC landing zone: kv_path 'direct', no byte on
the socket) and config 4 (a TP=2 engine over both ranks serving a wave) — with llama-mini shapes. Nothing here is a
scaling point; it proves the section runs and reports on a GPU."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_node_section_rehearsal_two_ranks_one_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--same-device", "--preset", "llama-mini", "--batch", "8",
           "--prompt-len", "64", "--gen-len", "16", "--max-model-len", "256", "--steps", "1", "--warmup", "1",
           "--tp-wave-min-world", "2", "--tp-wave-preset", "llama-mini", "--lb-preset", "mixtral-tiny",
           "--lb-kv-blocks", "64", "--lb-requests-per-worker", "8", "--cross-gpu-budget-s", "200", "--verbose"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=290)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    # a stall in the node section prints the line with the stalled part (watchdog, exit 3): show it
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    res = json.loads(lines[0])
    n = res["notes"]
    assert n["world_size_seen"] == 2 and n["distinct_devices"] == 1 and "rehearsal" in n
    cross = n["cross_gpu"]
    assert res["cross_gpu_status"] == "ok" and cross["status"] == 0, cross
    assert cross["xgpu_probe"]["kv_hop"]["per_rank"][1]["receiver_bytes_match"] is True, cross["xgpu_probe"]
    frp = cross["xgpu_probe"]["ipc_allreduce"]["fused_row_parallel"]["rehearsal"]  # fused vs separate one-shot
    assert frp["fused_us"] > 0 and frp["separate_one_shot_us"] > 0 and "half_ring" in frp, frp
    d = cross["disagg"]
    assert d["pairs"] == 1 and d["kv_path"] == "direct" and d["req_s_total"] > 0, d
    ab = d["per_pair"][0]["transport_ab"]  # shader stores (direct) vs copy engines (staged): both served
    assert ab["copy_engine_staged"]["req_s"] > 0 and ab["copy_engine_staged"]["staged_packets"] > 0, ab
    t = cross["tp_wave"]
    assert t["tp"] == 2 and t["all_tokens"] and t["graphs_replayed"] and t["error_word"] is False, t
    lb = cross["lb_serving"]  # config 5: a Mixtral worker per rank behind one coordinator
    assert lb["workers"] == 2 and [r["strategy"] for r in lb["runs"]] == ["least_latency", "round_robin"], lb
    assert all(r["requests"] == 16 and r["error_count"] == 0 for r in lb["runs"]), lb
