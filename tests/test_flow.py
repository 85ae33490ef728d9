"""Per-iteration flow ops: coords_grid_3d, upflow_3d and
RAFTDVC.forward's coords update + upsampling fused into one pass.

Reference: src/core/corr.py:71-99 (coords_grid_3d), :211-253 (upflow_3d),
src/core/raft_dvc.py:482-485 (coords1 = coords1 + delta_flow;
flow_up = upflow_3d(coords1 - coords0, target_shape)), :490 (log_b upsampling).

CPU: the float32 numpy oracle (oracle/oracle.py) against the reference's own outputs
(tests/golden/flow_*.npz, gen_flow_golden.py).  GPU: k_coords_grid / k_upflow through
the C ABI against the same fixtures and the oracle.  Tolerances:
  * coords_grid and coords1 + delta_flow: bit-exact (integers; one float32 add);
  * flow_up: max|out - ref| / max|ref| <= 1e-5 (SURVEY 8(c) fp32 bound; the GPU fuses
    the trilinear multiply-adds, so it differs from ATen's CPU loop by a few ulps).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle import oracle as orc

TOL = 1e-5
DEV = torch.device("cuda:0")
FLOW_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "flow_*.npz")))


def _case(name):
    import sys
    sys.path.insert(0, GOLDEN)
    import gen_flow_golden as gen
    g = load_golden(name + ".npz")
    B, h, w, d, H, W, D = (int(v) for v in g["shape"])
    c1, dl, lb = gen.flow_inputs(B, (h, w, d), float(g["max_flow"][0]), int(g["seed"][0]))
    return g, (B, h, w, d), (H, W, D), c1, dl, lb


def test_flow_fixtures_present():
    assert len(FLOW_CASES) >= 4


# ----------------------------------------------------------------------------- CPU: oracle vs reference
@pytest.mark.parametrize("name", FLOW_CASES)
def test_oracle_flow_against_reference(name):
    g, (B, h, w, d), tgt, c1, dl, lb = _case(name)
    hs = int(g["hstep"][0])
    assert np.array_equal(orc.coords_grid_3d(B, h, w, d), g["coords0"])
    new, up = orc.flow_step(c1, dl, tgt)
    assert np.array_equal(new, g["coords1"])
    assert orc.rel_err(up[:, :, ::hs], g["flow_up"]) <= 1e-6
    if "log_b_up" in g:
        assert orc.rel_err(orc.upflow_3d(lb, tgt), g["log_b_up"]) <= 1e-6
        up8 = orc.upflow_3d(new - g["coords0"], (8 * h, 8 * w, 8 * d))
        assert orc.rel_err(up8, g["up8"]) <= 1e-6


def test_flow_validation_without_gpu():
    """Argument errors raise before any launch (no GPU needed)."""
    import ctypes
    from dvccorr import _lib
    L = _lib.lib()
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    assert L.dvc_upflow(p, p, 1, 2, 2, 2, 2, 4, 4, 4, None) == _lib.DVC_ERR_INVALID       # C < 3
    assert L.dvc_upflow(None, p, 1, 3, 2, 2, 2, 4, 4, 4, None) == _lib.DVC_ERR_INVALID
    assert L.dvc_flow_step(p, None, None, p, 1, 2, 2, 2, 4, 4, 4, None) == _lib.DVC_ERR_INVALID  # up aliases coords1
    assert L.dvc_coords_grid(p, 1, 0, 2, 2, None) == _lib.DVC_ERR_INVALID
    L.dvc_flow_step(p, None, None, p, 1, 2, 2, 2, 4, 4, 4, None)
    assert b"alias" in L.dvc_last_error()
    with pytest.raises(RuntimeError):
        import dvccorr
        dvccorr.upflow_3d(torch.zeros(1, 3, 2, 2, 2), (4, 4, 4))


# ----------------------------------------------------------------------------- GPU: HIP vs reference / oracle
@pytest.mark.gpu
@pytest.mark.parametrize("name", FLOW_CASES)
def test_gpu_flow_step_against_reference(name):
    import dvccorr
    g, (B, h, w, d), tgt, c1, dl, lb = _case(name)
    hs = int(g["hstep"][0])
    grid = dvccorr.coords_grid_3d(B, h, w, d, DEV)
    assert np.array_equal(grid.cpu().numpy(), g["coords0"])
    c1_t = torch.from_numpy(c1).to(DEV)
    new, up = dvccorr.flow_step(c1_t, torch.from_numpy(dl).to(DEV), tgt)
    torch.cuda.synchronize()
    assert np.array_equal(new.cpu().numpy(), g["coords1"])
    assert np.array_equal(c1_t.cpu().numpy(), c1)          # input not modified
    assert up.shape == (B, 3, *tgt)
    assert orc.rel_err(up.cpu().numpy()[:, :, ::hs], g["flow_up"]) <= TOL
    # the unfused reference sequence on the GPU: upflow_3d(coords1 - coords0) agrees to rounding
    up2 = dvccorr.upflow_3d(new - grid, target_shape=tgt)
    assert orc.rel_err(up.cpu().numpy(), up2.cpu().numpy()) <= 1e-6
    if "log_b_up" in g:
        lb_up = dvccorr.upflow_3d(torch.from_numpy(lb).to(DEV), target_shape=tgt)
        assert orc.rel_err(lb_up.cpu().numpy(), g["log_b_up"]) <= TOL
        up8 = dvccorr.upflow_3d(new - grid)                # scale_factor=8 branch
        assert orc.rel_err(up8.cpu().numpy(), g["up8"]) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("B,lo,tgt", [
    (1, (32, 32, 32), (128, 128, 128)),   # cfg #3 iteration tail (1/4 encoder)
    (1, (16, 16, 16), (128, 128, 128)),   # cfg #2 (1/8 encoder)
    (2, (3, 5, 7), (3, 5, 7)),            # identity resize
    (1, (6, 4, 5), (2, 3, 9)),            # downsampling axes
    (1, (1, 1, 1), (4, 4, 4)),            # single source voxel
    (1, (5, 5, 5), (1, 1, 1)),            # single target voxel (ratio 0)
])
def test_gpu_flow_step_against_oracle(B, lo, tgt):
    import dvccorr
    import prng
    h, w, d = lo
    c1 = prng.flow_coords(700 + h, B, h, w, d, 4.0)
    dl = prng.uniform(701 + w, (B, 3, h, w, d), -1.5, 1.5)
    new, up = dvccorr.flow_step(torch.from_numpy(c1).to(DEV), torch.from_numpy(dl).to(DEV), tgt)
    onew, oup = orc.flow_step(c1, dl, tgt)
    assert np.array_equal(new.cpu().numpy(), onew)
    assert orc.rel_err(up.cpu().numpy(), oup) <= TOL
    # no delta: flow_up of coords1 - coords0 alone
    new0, up0 = dvccorr.flow_step(torch.from_numpy(c1).to(DEV), None, tgt)
    assert np.array_equal(new0.cpu().numpy(), c1)
    assert orc.rel_err(up0.cpu().numpy(), orc.flow_step(c1, None, tgt)[1]) <= TOL


@pytest.mark.gpu
def test_gpu_upflow_extra_channels_and_errors():
    """C > 3: channels 3.. are interpolated but not scaled (corr.py:249-251 scale 0..2 only)."""
    import dvccorr
    import prng
    x = prng.uniform(720, (1, 5, 4, 6, 3), -1, 1)
    up = dvccorr.upflow_3d(torch.from_numpy(x).to(DEV), target_shape=(8, 11, 9))
    assert orc.rel_err(up.cpu().numpy(), orc.upflow_3d(x, (8, 11, 9))) <= TOL
    with pytest.raises(ValueError):
        dvccorr.upflow_3d(torch.zeros(1, 2, 4, 4, 4, device=DEV), (8, 8, 8))
    with pytest.raises(ValueError):
        dvccorr.flow_step(torch.zeros(1, 3, 4, 4, 4, device=DEV), torch.zeros(1, 3, 4, 4, 2, device=DEV), (8, 8, 8))


@pytest.mark.gpu
@pytest.mark.parametrize("lo,tgt", [
    ((32, 32, 32), (128, 128, 128)),      # cfg #3 tail: 8 x-rows of 128 per 1024-output chunk
    ((64, 16, 24), (128, 64, 96)),        # x2 / x4 / x4 per axis
    ((20, 8, 12), (21, 16, 24)),          # ratio ~0.95 in h
    ((7, 5, 6), (7, 10, 12)),             # identity in h (ratio 1)
    ((4, 3, 700), (8, 5, 2048)),          # D > 1024: a chunk is part of one x row (z sub-range staged)
    ((40, 2, 3000), (44, 3, 4096)),       # rows >= 8: box bound above the LDS tile, the host takes the direct kernel
    ((6, 6, 6), (6, 6, 4)),               # downsampling in z: direct kernel (staged needs every ratio <= 1)
])
@pytest.mark.parametrize("rows", [1, 3, 8, 16])
def test_gpu_upflow_staged_matches_direct(lo, tgt, rows):
    """k_upflow's LDS-staged form (dvc_set_tuning "upflow_staged" 1, the default) and the direct
    per-lane gathers (0) compute the same T values in the same order: bitwise equal outputs."""
    import dvccorr
    import prng
    from dvccorr import _lib
    h, w, d = lo
    c1 = torch.from_numpy(prng.flow_coords(730 + h, 1, h, w, d, 3.0)).to(DEV)
    dl = torch.from_numpy(prng.uniform(731 + w, (1, 3, h, w, d), -1.0, 1.0)).to(DEV)
    outs = []
    try:
        _lib.set_tuning("upflow_rows", rows)
        for st in (0, 1):
            _lib.set_tuning("upflow_staged", st)
            outs.append(dvccorr.flow_step(c1, dl, tgt)[1])
    finally:
        _lib.set_tuning("upflow_staged", 1)
        _lib.set_tuning("upflow_rows", 12)   # the library default
    assert torch.equal(outs[0], outs[1])
    if rows == 8:
        assert orc.rel_err(outs[1].cpu().numpy(), orc.flow_step(c1.cpu().numpy(), dl.cpu().numpy(), tgt)[1]) <= TOL
