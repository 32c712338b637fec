"""bench/tp_probe.py on CPU: rank 0's shard of a TP=2 / TP=4 model runs the serving workload in one
process with the collectives stubbed (src/parallel/tp.py ShardProbeTP) — shard shapes, the
vocab-parallel LM head and the step loop all work without a process group."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("tp", [2, 4])
def test_tp_probe_runs_shard_on_cpu(tp):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "tp_probe.py"), "--preset", "llama-mini",
                        "--tp", str(tp), "--batch", "3", "--prompt-len", "20", "--gen-len", "5", "--steps", "1",
                        "--warmup", "0", "--device", "cpu"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["bench"] == "tp_shard_probe" and d["tp"] == tp and d["decode_ms_per_step"] > 0
    assert "all-reduce" in d["not_included"]


def test_decode_tile_table_keeps_statistics_tiles_within_the_consumers():
    """Mode 3 (residual update) writes one row-statistics tile per wr output columns; the fused attention
    prologue and the gate/up row scale read at most SSP_MAX_TILES (256) of them at <= 32 rows and
    SSP_MAX_TILES_WIDE (128) above — more would turn the whole fused decode path off."""
    from src import ops

    for (n, k, mode, bucket) in ops.DECODE_TILE_CFG:
        wr, kc, sk = ops.decode_tile(n, k, mode, bucket)
        if mode == 3:
            lim = ops.SSP_MAX_TILES if bucket <= 32 else ops.SSP_MAX_TILES_WIDE
            assert n // wr <= lim, (n, k, bucket, wr)
    # 70B TP=8 at <= 32 rows: wr = 32 tiles (256 of them) measured faster (profiles/r5_tp8_tiles_wr32.jsonl)
    assert ops.decode_tile(8192, 1024, 3, 32)[0] == 32 and ops.decode_tile(8192, 3584, 3, 32)[0] == 32
    assert ops.decode_tile(8192, 1024, 3, 64)[0] >= 64


def test_tile_override_parser():
    from src import ops

    assert ops._tile_overrides("4096,4096,3,32=32,256,2; 14336,4096,4,32=128,128,1") == {
        (4096, 4096, 3, 32): (32, 256, 2), (14336, 4096, 4, 32): (128, 128, 1)}


def test_tile_order_pack_unpack_round_trip():
    """ops.gd_pack_weights / gd_unpack_weights (the decode GEMM's tile order; the LM head is kept in it in
    place, and unpacked for checkpoint export and the fp32 reference copy) are exact inverses."""
    import torch

    from src import ops

    for wr, kc, rows, k in ((128, 128, 1024, 512), (64, 256, 640, 1024), (64, 128, 256, 4096), (32, 256, 96, 512)):
        w = torch.randn(rows, k).to(torch.bfloat16)
        p = ops.gd_pack_weights(w, wr, kc=kc)
        assert p.shape == w.shape and not torch.equal(p, w)
        assert torch.equal(ops.gd_unpack_weights(p, wr, kc=kc), w), (wr, kc)


def test_prefill_gemm_table_is_well_formed():
    """The shipped prefill GEMM table (src/ops/gemm_table.py): validators for the stack it was measured on,
    only TN bf16 entries with a named solution (no 'Default' rows: those shapes keep the library path), the
    Llama-3-8B bench wave's qkv / o / gate-up shapes present; loading it is a no-op without a GPU."""
    from src.ops import gemm_table

    lines = open(gemm_table.TABLE).read().splitlines()
    vals = {l.split(",")[1] for l in lines if l.startswith("Validator,")}
    assert {"PT_VERSION", "HIP_VERSION", "HIPBLASLT_VERSION", "GCN_ARCH_NAME", "ROCBLAS_VERSION"} <= vals
    assert any("gfx950" in l for l in lines if l.startswith("Validator,GCN_ARCH_NAME"))
    ent = gemm_table.table_entries()
    assert ent and all(s != "Default" for s in ent.values())
    for n, k in ((6144, 4096), (4096, 4096), (28672, 4096)):
        assert (n, 16384, k) in ent
    import torch

    if not torch.cuda.is_available():
        assert gemm_table.enable_prefill_gemm_table() is False
