"""GPU: the DVC_BRICKED pyramid layout (levels with >= 64-byte z-rows in (1, 8, 8) bricks of one 128-byte
line, include/dvccorr.h).  The bricked pack is the linear pack permuted; the lookups on a bricked pyramid are
bit-identical to the same lookups on the linear one (same values, same arithmetic, only the addresses move);
the reference-shaped pyramid views gather bricked levels back; the linear-only entry points refuse it."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _inputs(shape, C, B=1, flow=3.0, seed=0):
    import dvccorr
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(seed + H * 7 + W * 3 + D + C)
    f1 = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    c = dvccorr.coords_grid_3d(B, H, W, D, torch.device("cpu")) + (torch.rand(B, 3, H, W, D, generator=g) * 2 - 1) * flow
    c.view(B, 3, -1)[:, :, 3] = float("nan")
    c.view(B, 3, -1)[:, 1, 11] = 1e30
    return f1, f2, c.to(DEV)


@pytest.mark.parametrize("shape,C,L", [((32, 32, 32), 64, 4), ((40, 48, 40), 32, 3), ((64, 64, 64), 32, 2)])
@pytest.mark.parametrize("prec", ["bf16", "fp32"])
def test_bricked_pack_is_a_permutation(shape, C, L, prec):
    from dvccorr import ops
    from dvccorr.corr_block import brick_index
    H, W, D = shape
    f2 = torch.randn(2, C, H, W, D, device=DEV)
    dt = ops.dtype_code(prec)
    lin = ops.pack_targets(f2, L, dt)
    brk = torch.full_like(lin, float("nan"))
    ops.pack_targets(f2, L, dt | ops.DVC_BRICKED, out=brk)
    lay = ops.layout(H, W, D, L, C)
    mask = ops.bricked_levels(lay)
    assert mask != 0
    want = lin.clone()
    for l, (h, w, d) in enumerate(lay.levels()):
        if (mask >> l) & 1:
            off, n = lay.offset[l], h * w * lay.Dp[l]
            want[:, off + brick_index(h, w, lay.Dp[l], DEV)] = lin[:, off:off + n]
    torch.cuda.synchronize()
    assert torch.equal(brk, want)


@pytest.mark.parametrize("shape,C,L,r,legacy,B", [
    ((32, 32, 32), 128, 4, 4, False, 1),    # config #3 shape
    ((24, 32, 40), 64, 3, 3, False, 2),     # non-cubic, ragged tiles, two batch elements
    ((16, 40, 40), 32, 2, 4, True, 1),      # legacy with W == D on the bricked level
    ((32, 24, 64), 32, 4, 1, False, 1),     # r = 1
    ((20, 32, 33), 32, 3, 6, False, 1),     # r = 6, D padded to 40
])
@pytest.mark.parametrize("prec", ["bf16", "fp32"])
def test_bricked_lookup_bitwise_equal(shape, C, L, r, legacy, B, prec):
    import dvccorr
    f1, f2, c = _inputs(shape, C, B)
    with torch.no_grad():
        lin = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision=prec, bricked=False)
        brk = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision=prec)
        assert brk._brick and not lin._brick
        a, b = lin(c), brk(c)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        for pl, pb in zip(lin.corr_pyramid, brk.corr_pyramid):
            assert torch.equal(pl, pb)
        if r <= 4:
            K = L * (2 * r + 1) ** 3
            w = (torch.rand(96, K, device=DEV) * 2 - 1) / K ** 0.5
            bias = (torch.rand(96, device=DEV) * 2 - 1) / K ** 0.5
            assert torch.equal(lin.lookup_convc1(c, w, bias), brk.lookup_convc1(c, w, bias))


def test_bricked_slab_rows():
    """One rank's H-slab (HipRows, the sharded/bench path): bricked rows give the same lookup as linear rows,
    on the row-split launch of a small slab too."""
    import os
    from dvccorr.sharded import HipRows
    S, C, L, r = 32, 128, 4, 4
    f1, f2, c = _inputs((S, S, S), C)
    q = f1[:, :, 8:12].reshape(1, C, -1).contiguous()
    cf = c[:, :, 8:12].reshape(1, 3, -1).contiguous()
    with torch.no_grad():
        rows = HipRows(q, f2, L, r, False, "bf16", "materialised")
        assert rows.ldt != rows.dt
        os.environ["DVCCORR_BRICKED"] = "0"
        try:
            lin = HipRows(q, f2, L, r, False, "bf16", "materialised")
        finally:
            del os.environ["DVCCORR_BRICKED"]
        assert lin.ldt == lin.dt
        assert torch.equal(rows.lookup(cf), lin.lookup(cf))


def test_bricked_refused_where_linear():
    """Entry points that read the linear layout refuse DVC_BRICKED instead of misreading it."""
    from dvccorr import _lib, ops
    S, C, L = 32, 32, 4
    f1, f2, c = _inputs((S, S, S), C)
    dt = ops.dtype_code("bf16")
    t = ops.pack_targets(f2, L, dt | ops.DVC_BRICKED)
    q = ops.pack_queries(f1.reshape(1, C, -1), dt)
    corr = ops.build(q, t, C, S, S, S, L, dt, dt)
    cf = c.reshape(1, 3, -1)
    with pytest.raises(ValueError, match="bad dtype"):            # the pool reads the linear layout
        ops.pool(corr, S, S, S, L, 0, dt | ops.DVC_BRICKED)
    with pytest.raises(ValueError, match="dtype"):                # the build is layout-blind: plain dtypes only
        ops.build(q, t, C, S, S, S, L, dt | ops.DVC_BRICKED, dt)
    _lib.set_tuning("lookup_variant", 0)
    try:
        with pytest.raises(NotImplementedError, match="tile kernel"):
            ops.lookup(corr, cf, S, S, S, L, 4, False, dt | ops.DVC_BRICKED)
    finally:
        _lib.set_tuning("lookup_variant", 2)
    with pytest.raises(NotImplementedError, match="tile kernel"):   # radius 7: the walk
        ops.lookup(corr, cf, S, S, S, L, 7, False, dt | ops.DVC_BRICKED)
    with pytest.raises(NotImplementedError, match="single-pass"):
        ops.pack_targets(torch.randn(1, C, S, S, S, device=DEV), 5, dt | ops.DVC_BRICKED)
    # the C ABI cannot tell a bricked buffer from a linear one; the Python layer records the flag
    with pytest.raises(ValueError, match="packed bricked"):
        ops.lookup(corr, cf, S, S, S, L, 4, False, dt)
    with pytest.raises(ValueError, match="packed bricked"):
        ops.lookup_fused(q, t, cf, C, S, S, S, L, 4, False, dt)
    with pytest.raises(ValueError, match="packed bricked"):
        ops.corr_backward(q, t, cf, torch.zeros(1, L * 729, S ** 3, device=DEV), C, S, S, S, L, 4, False, dt)
    torch.cuda.synchronize()
