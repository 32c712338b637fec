"""Prefill GEMM selection from a tuned table (PyTorch TunableOp over hipBLASLt + rocBLAS).

The prefill projections (M = thousands of tokens) run on hipBLASLt/rocBLAS through
``torch.nn.functional.linear``. The default heuristic leaves 15-30 % on the table on some
Llama shapes; ``scripts/tune_gemms.py`` times every solution of both libraries on an MI355X
and writes the winners to ``configs/tunableop_results_gfx950.csv`` (validators pin the
PyTorch / ROCm / hipBLASLt / rocBLAS versions and the gfx950 arch: a mismatching table is
ignored by TunableOp). At engine start this module loads the table with tuning itself
disabled, so no timing happens on the serving path; shapes not in the table use the
library default.

Measured (profiles/bench_r1_v6.log vs the tuned run): the table's winners were timed by
TunableOp in isolation and did not beat the default heuristic inside the bench (prefill GEMM
time 300 ms -> 303 ms per 2 waves), so it is opt-in: DIE_TUNED_GEMMS=1.
"""

from __future__ import annotations

import logging
import os
import tempfile

import torch

logger = logging.getLogger(__name__)

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "configs",
                     "tunableop_results_gfx950.csv")
_loaded = False


def enable_tuned_gemms(path: str = TABLE) -> bool:
    """Idempotent. Returns True when a tuned table is active."""
    global _loaded
    if _loaded:
        return True
    if os.environ.get("DIE_TUNED_GEMMS", "0") != "1" or not torch.cuda.is_available() or not os.path.exists(path):
        return False
    tun = torch.cuda.tunable
    try:
        tun.enable(True)
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        # anything TunableOp writes at exit goes to a private scratch file, never the shipped table
        tun.set_filename(os.path.join(tempfile.gettempdir(), f"die_tunableop_{os.getpid()}.csv"),
                         insert_device_ordinal=False)
        ok = tun.read_file(path)
    except Exception as e:  # pragma: no cover - depends on the torch build
        logger.warning("tuned GEMM table not loaded: %s", e)
        tun.enable(False)
        return False
    _loaded = bool(ok)
    if not _loaded:
        tun.enable(False)
    logger.info("tuned GEMM table %s: %s", path, "loaded" if _loaded else "rejected (validator mismatch)")
    return _loaded
