"""CPU checks of the host layer added in round 2 (no GPU needed):

  * the torch.library operators are registered with fake (meta) implementations that give the
    reference's output shapes (corr.py:169-208: (B, L*(2r+1)^3, N) float32), so they trace under
    FakeTensorMode / torch.compile, and dvccorr::lookup_ad carries an autograd formula with the
    fmap shapes and dtypes;
  * the adjoint used by the differentiable flow_step / upflow_3d equals autograd through the
    reference's upflow_3d formula (corr.py:211-253) on CPU tensors;
  * error paths that must fire before any GPU work (capacity arithmetic, backward support).
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F
from torch._subclasses.fake_tensor import FakeTensorMode

import dvccorr
from dvccorr import corr_block, library  # noqa: F401  (registers the ops)


def test_ops_registered_with_fake_shapes():
    B, C, H, W, D, L, r = 2, 64, 8, 9, 10, 3, 2
    lay = dvccorr.layout(H, W, D, L, C)
    n3 = (2 * r + 1) ** 3
    with FakeTensorMode():
        q = torch.empty(B, H * W * D, lay.c_pad, dtype=torch.bfloat16, device="cuda")
        t = torch.empty(B, lay.row_stride, lay.c_pad, dtype=torch.bfloat16, device="cuda")
        c = torch.empty(B, 3, H * W * D, device="cuda")
        corr = torch.ops.dvccorr.build(q, t, C, H, W, D, L, 1)
        assert corr.shape == (B, H * W * D, lay.row_stride) and corr.dtype == torch.bfloat16
        out = torch.ops.dvccorr.lookup(corr, c, H, W, D, L, r, False, 1)
        assert out.shape == (B, L * n3, H * W * D) and out.dtype == torch.float32
        out = torch.ops.dvccorr.lookup_fused(q, t, c, C, H, W, D, L, r, True, 1)
        assert out.shape == (B, L * n3, H * W * D) and out.dtype == torch.float32
        g = torch.empty(B, L * n3, H * W * D, device="cuda")
        d1, d2 = torch.ops.dvccorr.corr_backward(q, t, c, g, C, H, W, D, L, r, False, 1)
        assert d1.shape == (B, C, H * W * D) and d2.shape == (B, C, H, W, D)
        wp = torch.empty(1024, dtype=torch.float16, device="cuda")
        bias = torch.empty(96, device="cuda")
        out = torch.ops.dvccorr.lookup_fused_proj(q, t, c, wp, bias, C, H, W, D, L, r, False, 1)
        assert out.shape == (B, 96, H * W * D) and out.dtype == torch.float32


def test_lookup_ad_autograd_shapes():
    """dvccorr::lookup_ad's registered backward returns d fmap1 / d fmap2 in the fmaps' shapes and dtypes
    (traced with fake tensors: no kernel runs)."""
    B, C, H, W, D, L, r = 1, 32, 6, 7, 8, 2, 2
    lay = dvccorr.layout(H, W, D, L, C)
    # meta tensors: the registered fake implementation runs, and the autograd engine needs no device
    f1 = torch.empty(B, C, H, W, D, device="meta", dtype=torch.float16, requires_grad=True)
    f2 = torch.empty(B, C, H, W, D, device="meta", requires_grad=True)
    q = torch.empty(B, H * W * D, lay.c_pad, dtype=torch.bfloat16, device="meta")
    t = torch.empty(B, lay.row_stride, lay.c_pad, dtype=torch.bfloat16, device="meta")
    c = torch.empty(B, 3, H * W * D, device="meta")
    out = torch.ops.dvccorr.lookup_ad(f1, f2, None, q, t, c, C, H, W, D, L, r, False, 1)
    assert out.shape == (B, L * (2 * r + 1) ** 3, H * W * D)
    out.sum().backward()
    assert f1.grad.shape == f1.shape and f1.grad.dtype == torch.float16
    assert f2.grad.shape == f2.shape and f2.grad.dtype == torch.float32


@pytest.mark.parametrize("lo,hi", [((4, 5, 6), (16, 20, 24)), ((8, 8, 8), (64, 64, 64)), ((3, 1, 5), (9, 4, 15))])
def test_upflow_adjoint_matches_reference_autograd(lo, hi):
    g = torch.Generator().manual_seed(sum(lo))
    flow = torch.randn(2, 3, *lo, generator=g, requires_grad=True)
    up = F.interpolate(flow, size=hi, mode="trilinear", align_corners=True)   # corr.py:234-239
    scale = torch.tensor([hi[0] / lo[0], hi[1] / lo[1], hi[2] / lo[2]]).view(1, 3, 1, 1, 1)
    gu = torch.randn(2, 3, *hi, generator=g)
    (up * scale * gu).sum().backward()
    adj = corr_block._upflow_adjoint(gu, tuple(flow.shape))
    torch.testing.assert_close(adj, flow.grad, rtol=1e-5, atol=1e-5)


def test_backward_support_checked_at_construction():
    # any C: the gradient kernels run per 128-channel group (round 3; C = 256 trains like C = 128)
    corr_block._check_backward_support(dvccorr.layout(8, 8, 8, 2, 256), 256, 4, False)
    with pytest.raises(NotImplementedError, match="radius"):
        corr_block._check_backward_support(dvccorr.layout(8, 8, 8, 2, 64), 64, 7, False)


def test_pyramid_bytes():
    # 64^3 x 4 levels bf16 (config #4): 262144 rows x row_stride x 2 B = the 157 GB of SURVEY 8
    b = corr_block.pyramid_bytes(1, 128, 64, 64, 64, 4, "bf16")
    assert 155e9 < b < 160e9
    assert corr_block.pyramid_bytes(1, 128, 64, 64, 64, 4, "fp32") > 2 * b - 1024
