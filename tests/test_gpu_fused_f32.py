"""GPU: the fp32 on-the-fly block on the matrix cores (round 6, k_fused_box_f32 in
raft-dvc_amd/csrc/fused_box_f32.hip).

The reference's evaluation runs CorrBlockOnTheFly in fp32 (src/core/raft_dvc.py:403-412, the einsum at
src/core/corr_otf.py:237).  dvccorr's fp32 on-the-fly lookup takes its window dots on
v_mfma_f32_16x16x32_bf16 with both operands split into bf16 hi + lo (three MFMAs per step), keeps them in
fp32 and interpolates them with the tile lookup's arithmetic.  Held to the fp32 tolerance (1e-5 of the
output's max magnitude) against the fp32 materialised block (exact f32 MFMA build) and the
two-stage VALU path it replaces (fused_variant 0); the golden equiv_* / edge_* vectors run through it in
test_gpu_parity.py::test_small_cases_fp32[fused-*] and config #5's rows against the f64 oracle in
test_gpu_scale.py::test_cfg5_fused_rows[fp32-*].
"""
from __future__ import annotations

import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
FP32_TOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _no_grad():
    with torch.no_grad():
        yield


def _inputs(shape, C, r, seed, spread=None):
    import dvccorr
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(seed)
    f1 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    base = dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu"))
    c = base + (torch.rand(1, 3, H, W, D, generator=g) * 2 - 1) * (r + 6 if spread is None else spread)
    return f1, f2, c


@pytest.mark.parametrize("shape,C,L,r", [((9, 7, 5), 32, 2, 1), ((12, 10, 16), 64, 3, 2), ((16, 16, 16), 32, 4, 3),
                                         ((20, 13, 24), 128, 3, 4), ((32, 32, 32), 128, 4, 4),
                                         ((18, 34, 40), 64, 2, 4), ((8, 8, 8), 128, 2, 3)])
def test_fp32_fused_mfma_matches_materialised(shape, C, L, r):
    """Ragged query boxes, non-cubic sizes, flows wide enough to push the union past one z block and the window
    planes' two passes past the level, NaN / huge coordinates, both conventions (legacy W != D levels run the
    per-output kernel, as before): the matrix-core fp32 lookup within 1e-5 of the fp32 materialised block and of
    the VALU two-stage path; out-of-range queries give the same exact zeros."""
    import dvccorr
    from dvccorr import _lib
    f1, f2, c = _inputs(shape, C, r, shape[0] * 1000 + shape[1] * 10 + shape[2] + r + C)
    c.view(3, -1)[:, 5] = float("nan")
    c.view(3, -1)[1, 17] = 1e30
    c.view(3, -1)[2, 23] = -float("inf")
    c = c.to(DEV)
    for legacy in (False, True):
        ref = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision="fp32")(c)
        fz = dvccorr.CorrBlockFused(f1, f2, L, r, legacy_wd_swap=legacy, precision="fp32")
        try:
            _lib.set_tuning("fused_variant", 0)
            valu = fz(c)
            _lib.set_tuning("fused_variant", 2)
            out = fz(c)
            again = fz(c)
            torch.cuda.synchronize()
        finally:
            _lib.set_tuning("fused_variant", 2)
        assert torch.isfinite(out).all(), (shape, legacy)
        assert torch.equal(out, again), "not repeatable"
        e_ref = orc.rel_err(out.cpu().numpy(), ref.cpu().numpy())
        e_valu = orc.rel_err(out.cpu().numpy(), valu.cpu().numpy())
        assert e_ref <= FP32_TOL and e_valu <= FP32_TOL, (shape, C, L, r, legacy, e_ref, e_valu)
        # the dead queries' outputs are exact zeros, as the reference's grid_sample gives
        flat = out.reshape(out.shape[0], out.shape[1], -1)
        for qd in (5, 17, 23):
            assert not bool(flat[:, :, qd].any()), qd


def test_fp32_fused_bench_shape_and_slab():
    """Config #3's shape (32^3 x 128, L = 4, r = 4, +-2-voxel flows) at 1e-5 of the fp32 materialised block, and one
    rank's H-slab of queries (the sharded on-the-fly layout, dvccorr.sharded.HipRows) equal to that slab of the
    whole-grid result bit for bit."""
    import dvccorr
    from dvccorr.sharded import HipRows
    S, C, L, r = 32, 128, 4, 4
    f1, f2, c = _inputs((S, S, S), C, r, 3131, spread=2.0)
    c = c.to(DEV)
    ref = dvccorr.CorrBlock(f1, f2, L, r, precision="fp32")(c)
    out = dvccorr.CorrBlockFused(f1, f2, L, r, precision="fp32")(c)
    e = orc.rel_err(out.cpu().numpy(), ref.cpu().numpy())
    assert e <= FP32_TOL, e
    full = out.reshape(1, L * (2 * r + 1) ** 3, -1)
    h0, h1 = 8, 12
    part = HipRows(f1[:, :, h0:h1].reshape(1, C, -1), f2, L, r, False, "fp32", "fused").lookup(
        c[:, :, h0:h1].reshape(1, 3, -1).contiguous())
    assert torch.equal(part, full[:, :, h0 * S * S:h1 * S * S])


def test_fp32_fused_batch2():
    """Two batch elements with different features and flows: each item within 1e-5 of its own materialised result
    (a batch-offset error in the split operands cannot hide behind the other item's scale)."""
    import dvccorr
    H, W, D, C, L, r = 12, 10, 16, 64, 3, 4
    g = torch.Generator(device="cpu").manual_seed(2121)
    f1 = torch.randn(2, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(2, C, H, W, D, generator=g).to(DEV)
    c = (dvccorr.coords_grid_3d(2, H, W, D, torch.device("cpu")) +
         (torch.rand(2, 3, H, W, D, generator=g) * 2 - 1) * 5).to(DEV)
    ref = dvccorr.CorrBlock(f1, f2, L, r, precision="fp32")(c)
    out = dvccorr.CorrBlockFused(f1, f2, L, r, precision="fp32")(c)
    for b in range(2):
        e = orc.rel_err(out[b].cpu().numpy(), ref[b].cpu().numpy())
        assert e <= FP32_TOL, (b, e)
