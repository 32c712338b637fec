"""CPU paths of the prefill row-scale ops (the GPU kernels are checked in tests/test_kernels_gpu.py)."""

import torch

from src import ops


def test_linear_residual_adds_in_place():
    torch.manual_seed(0)
    res = torch.randn(37, 64)
    x = torch.randn(37, 96)
    w = torch.randn(64, 96) / 10
    want = res + x @ w.t()
    ptr = res.data_ptr()
    out = ops.linear_residual(res, x, w)
    assert out.data_ptr() == ptr
    torch.testing.assert_close(res, want, rtol=1e-5, atol=1e-5)


def test_linear_residual_on_row_blocks():
    """Row views of the residual (a chunked prefill's token blocks) are updated in place, the rest untouched."""
    torch.manual_seed(1)
    res = torch.randn(40, 32)
    keep = res.clone()
    x = torch.randn(16, 48)
    w = torch.randn(32, 48) / 8
    ops.linear_residual(res[8:24], x, w)
    torch.testing.assert_close(res[8:24], keep[8:24] + x @ w.t(), rtol=1e-5, atol=1e-5)
    assert torch.equal(res[:8], keep[:8]) and torch.equal(res[24:], keep[24:])


def test_rms_row_scale_stats_only_leaves_residual():
    torch.manual_seed(2)
    res = torch.randn(9, 128)
    keep = res.clone()
    rs = ops.rms_row_scale(res, None, 1e-5)
    assert torch.equal(res, keep)
    torch.testing.assert_close(rs, torch.rsqrt(keep.pow(2).mean(-1) + 1e-5))


def test_attention_part_policy_switch_is_safe_without_a_gpu():
    ops.set_attn_few_pair_parts(False)
    ops.set_attn_few_pair_parts(True)
