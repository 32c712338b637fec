"""A/B helper: bench.py with the prefill GEMM table read from another CSV (argv[1]); the rest of argv goes to
bench.py. enable_prefill_gemm_table binds its path default at definition, so the default is replaced."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import src.ops.gemm_table as gt  # noqa: E402

path = os.path.abspath(sys.argv[1])
_enable = gt.enable_prefill_gemm_table
gt.enable_prefill_gemm_table = lambda device=None, path=path: _enable(device, path)
gt.TABLE = path

import bench  # noqa: E402

sys.exit(bench.main(sys.argv[2:]))
