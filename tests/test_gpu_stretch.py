"""Legacy sampler levels with W != D (reference corr.py:49-52, legacy_wd_swap): k_lookup_stretch (round 6, LDS-staged
stretched boxes) against k_lookup_generic (per-output gathers, tuning lookup_stretch 0) -- bit for bit, since both
evaluate tri_sample's arithmetic in its term order -- and against the CPU oracle (fp32, <= 1e-5 of max|ref|)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _no_grad():
    with torch.no_grad():
        yield


def _lookup(f1, f2, coords, L, r, precision, stretch):
    import dvccorr
    from dvccorr import _lib
    _lib.set_tuning("lookup_stretch", stretch)
    try:
        blk = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=True, precision=precision)
        out = blk(coords)
        torch.cuda.synchronize()
        return out
    finally:
        _lib.set_tuning("lookup_stretch", 1)


def _inputs(B, C, H, W, D, flow, seed, specials=False):
    import dvccorr
    g = torch.Generator(device="cpu").manual_seed(seed)
    f1 = torch.randn(B, C, H, W, D, generator=g)
    f2 = torch.randn(B, C, H, W, D, generator=g)
    c = dvccorr.coords_grid_3d(B, H, W, D, torch.device("cpu")) + (torch.rand(B, 3, H, W, D, generator=g) * 2 - 1) * flow
    if specials:   # NaN, +-inf, huge, far outside: every corner out of range -> 0, as grid_sample's zero padding
        flat = c.view(B, 3, -1)
        flat[0, 0, 0] = float("nan")
        flat[0, 2, 1] = float("inf")
        flat[0, 1, 2] = -3.0e7
        flat[0, 2, 3] = 5.0e6
        flat[-1, 1, -1] = -40.0
    return f1.to(DEV), f2.to(DEV), c.to(DEV)


SHAPES = [((12, 16, 8), 3), ((10, 6, 14), 2), ((8, 24, 6), 2), ((9, 7, 20), 2), ((16, 8, 16), 4)]


@pytest.mark.parametrize("precision", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape,L", SHAPES)
def test_stretch_matches_generic_bitwise(shape, L, precision):
    H, W, D = shape
    for r in (1, 4, 6) if precision == "bf16" else (4,):
        f1, f2, c = _inputs(2, 32, H, W, D, 3.0, seed=H * 100 + W + r, specials=True)
        a = _lookup(f1, f2, c, L, r, precision, 1)
        b = _lookup(f1, f2, c, L, r, precision, 0)
        assert torch.isfinite(a).all()
        assert torch.equal(a, b), (shape, L, r, precision, float((a - b).abs().max()))


@pytest.mark.parametrize("r", [2, 3, 5])
def test_stretch_radii_ragged(r):
    # 7 x 10 x 5 = 350 queries: a ragged last tile of each batch element
    f1, f2, c = _inputs(1, 64, 7, 10, 5, 2.5, seed=40 + r)
    a = _lookup(f1, f2, c, 2, r, "bf16", 1)
    b = _lookup(f1, f2, c, 2, r, "bf16", 0)
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape,L", [((6, 10, 4), 2), ((5, 4, 9), 2)])
def test_stretch_against_oracle(shape, L):
    H, W, D = shape
    f1, f2, c = _inputs(1, 16, H, W, D, 2.0, seed=7)
    out = _lookup(f1, f2, c, L, 4, "fp32", 1).cpu().numpy()
    ref = orc.corr_lookup(f1.cpu().numpy().astype(np.float64), f2.cpu().numpy().astype(np.float64),
                          c.cpu().numpy().astype(np.float64), L, 4, True)
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert err <= 1e-5, err


def _lookup_fused(f1, f2, coords, L, r, precision, stretch):
    import dvccorr
    from dvccorr import _lib
    _lib.set_tuning("lookup_stretch", stretch)
    try:
        out = dvccorr.CorrBlockFused(f1, f2, L, r, legacy_wd_swap=True, precision=precision)(coords)
        torch.cuda.synchronize()
        return out
    finally:
        _lib.set_tuning("lookup_stretch", 1)


@pytest.mark.parametrize("precision", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape,L", [((12, 16, 8), 3), ((9, 7, 20), 2), ((16, 8, 16), 4)])
def test_fused_stretch_matches_generic_bitwise(shape, L, precision):
    """On the fly: window-box dots + k_lookup_stretch<WINBUF> against k_fused_generic's per-output corner dots."""
    H, W, D = shape
    for r in (2, 4) if precision == "bf16" else (4,):
        f1, f2, c = _inputs(2, 32, H, W, D, 3.0, seed=H * 10 + W + D + r, specials=True)
        a = _lookup_fused(f1, f2, c, L, r, precision, 1)
        b = _lookup_fused(f1, f2, c, L, r, precision, 0)
        assert torch.isfinite(a).all()
        assert torch.equal(a, b), (shape, L, r, precision, float((a - b).abs().max()))


def test_fused_stretch_against_materialised_fp32():
    """fp32 on the fly (exact dots) against the fp32 materialised block on legacy W != D levels: <= 1e-5."""
    f1, f2, c = _inputs(1, 32, 10, 6, 14, 2.0, seed=3)
    a = _lookup_fused(f1, f2, c, 2, 4, "fp32", 1)
    b = _lookup(f1, f2, c, 2, 4, "fp32", 1)
    err = float((a - b).abs().max() / b.abs().max())
    assert err <= 1e-5, err


def _backward(f1, f2, coords, L, r, precision, stretch):
    from dvccorr import _lib, ops
    B, C, H, W, D = f1.shape
    dt = ops.dtype_code(precision)
    q = ops.pack_queries(f1.reshape(B, C, -1), dt)
    t = ops.pack_targets(f2, L, dt)
    g = torch.Generator(device=DEV).manual_seed(5)
    gout = torch.randn(B, L * (2 * r + 1) ** 3, H * W * D, device=DEV, generator=g)
    _lib.set_tuning("bwd_stretch", stretch)
    try:
        d1, d2 = ops.corr_backward(q, t, coords.reshape(B, 3, -1).contiguous(), gout, C, H, W, D, L, r, True, dt)
        torch.cuda.synchronize()
        return d1, d2
    finally:
        _lib.set_tuning("bwd_stretch", 1)


@pytest.mark.parametrize("precision", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape,L", [((12, 16, 8), 3), ((9, 7, 20), 2), ((16, 8, 16), 4), ((8, 24, 6), 2)])
def test_backward_stretch_matches_generic_bitwise(shape, L, precision):
    """Legacy W != D window gradients: k_win_grad_stretch (LDS planes) against k_win_grad_generic (global boxes)."""
    H, W, D = shape
    for r in (1, 4) if precision == "bf16" else (4,):
        f1, f2, c = _inputs(2, 32, H, W, D, 3.0, seed=H + W * 7 + D + r, specials=True)
        a1, a2 = _backward(f1, f2, c, L, r, precision, 1)
        b1, b2 = _backward(f1, f2, c, L, r, precision, 0)
        assert torch.isfinite(a1).all() and torch.isfinite(a2).all()
        assert torch.equal(a1, b1) and torch.equal(a2, b2), (shape, L, r, precision)


def test_stretch_too_wide_falls_back():
    """A stretch whose staged boxes would need more than 64 KB of LDS per wave (W-1 = 21 (D-1) here) keeps the
    generic kernels; the result is the same either way."""
    f1, f2, c = _inputs(1, 32, 6, 64, 4, 2.0, seed=9)
    a = _lookup(f1, f2, c, 1, 4, "bf16", 1)
    b = _lookup(f1, f2, c, 1, 4, "bf16", 0)
    assert torch.equal(a, b)
    fa = _lookup_fused(f1, f2, c, 1, 4, "bf16", 1)
    fb = _lookup_fused(f1, f2, c, 1, 4, "bf16", 0)
    assert torch.equal(fa, fb)
    ga = _backward(f1, f2, c, 1, 4, "bf16", 1)
    gb = _backward(f1, f2, c, 1, 4, "bf16", 0)
    assert torch.equal(ga[0], gb[0]) and torch.equal(ga[1], gb[1])
