"""Prefill GEMM solution table (PyTorch TunableOp, read-only).

Prefill projections (M in the thousands) run on the ROCm libraries through ``torch.nn.functional.linear``.
The libraries' default heuristic is not always their fastest solution at the serving shapes:
``bench/micro_prefill_tunableop.py`` times every hipBLASLt and rocBLAS solution for the dense Llama-3 prefill
shapes (8B, its TP=2 shard, the 70B TP=8 shard; 2,048-16,384 tokens per step) on MI355X, and the entries whose
winner beat the default by >= 3 % in our own event timing (random bf16 operands) are kept in
``gemm_table_gfx950.csv`` (e.g. Llama-3-8B at 16,384 tokens: qkv 1.19x, o 1.08x, gate/up 1.04x;
profiles/r5_prefill_gemm_table.jsonl). At engine start the table is loaded with tuning OFF: a listed shape uses
its recorded solution, every other GEMM the default path — no timing ever happens in a serving process. The
table's validators (PyTorch, HIP, hipBLASLt, rocBLAS versions, gfx950) must match the running stack, else
PyTorch rejects it and the defaults stay.
"""
import logging
import os

import torch

logger = logging.getLogger(__name__)

TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_table_gfx950.csv")
_loaded = None


def table_entries(path: str = TABLE) -> dict:
    """{(N, M, K): solution} of the table's TN bf16 GEMM entries (x [M, K] @ w[N, K]^T)."""
    out = {}
    with open(path) as f:
        for line in f:
            parts = line.strip().split(",")
            if len(parts) == 4 and parts[0] == "GemmTunableOp_BFloat16_TN":
                dims = parts[1].split("_")
                out[(int(dims[1]), int(dims[2]), int(dims[3]))] = parts[2]
    return out


def warm_table(device, path: str = TABLE) -> None:
    """Run every listed GEMM once on ``device`` (operands uninitialised; results discarded). The table names
    rocBLAS as well as hipBLASLt solutions: the first call into a library (handle creation, code-object
    loads) can take a second or more, and a tensor-parallel rank that pays it inside its first prefill step
    while its peers already wait in a one-shot collective would trip their bounded wait (a spurious TP fault).
    Paying it here, before serving, keeps the first prefill step as fast as the others."""
    for (n, m, k) in sorted(table_entries(path), key=lambda e: e[0] * e[1] * e[2]):
        x = torch.empty(m, k, dtype=torch.bfloat16, device=device)
        w = torch.empty(n, k, dtype=torch.bfloat16, device=device)
        torch.nn.functional.linear(x, w)
        del x, w
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()


def enable_prefill_gemm_table(device=None, path: str = TABLE) -> bool:
    """Load the table read-only into PyTorch TunableOp (once per process) and warm its libraries on ``device``
    (default: the current device). Returns whether it is active."""
    global _loaded
    if _loaded is not None:
        return _loaded
    _loaded = False
    if not (torch.cuda.is_available() and torch.version.hip and os.path.exists(path)):
        return False
    try:
        import torch.cuda.tunable as tun

        tun.enable(True)
        tun.tuning_enable(False)          # never time anything in a serving process
        tun.record_untuned_enable(False)
        _loaded = bool(tun.read_file(path))
        if not _loaded:
            tun.enable(False)
        else:
            warm_table(device if device is not None else torch.device("cuda", torch.cuda.current_device()), path)
    except Exception as e:  # a stack the table was not made on: keep the library defaults
        logger.warning("prefill GEMM table not loaded: %s", e)
        _loaded = False
    return _loaded
