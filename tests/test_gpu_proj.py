"""GPU parity of the convc1-fused lookup (dvc_corr_lookup_proj, CorrBlock.lookup_convc1).

Reference: CorrBlock.__call__ (src/core/corr.py:169-208) followed by MotionEncoder's
F.relu(self.convc1(corr)) (src/core/update.py:219-222, 246).  On a bf16 block the fused kernel
feeds the lookup values and the weights to fp16 MFMA with fp32 accumulation (as the reference's
AMP convc1 runs in fp16), so the tolerance is the bf16 one of SURVEY.md 8(c): max|out - ref| /
max|ref| <= 1e-2; an fp32 block (round 5) runs the exact split consumer -- lookup values and weights as bf16
hi + lo, three MFMAs per step -- at the fp32 tolerance 1e-5.  Against
  * the reference's own outputs (tests/golden/proj_*.npz, gen_proj_golden.py),
  * the CPU oracle (f64 lookup + motion_convc1) on ragged / non-cubic / zero-level cases,
  * the unfused GPU composition relu(conv3d(lookup)) at the bench size (32^3, C=128, L=4, r=4).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch

import prng
from conftest import GOLDEN, load_golden, proj_inputs
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

PROJ_TOL = 1e-2
FP32_TOL = 1e-5
FUSED_VS_UNFUSED_TOL = 2e-3
DEV = torch.device("cuda:0")
PROJ_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "proj_*.npz")))


@pytest.fixture(scope="module", autouse=True)
def _no_grad():
    with torch.no_grad():
        yield


def _gpu(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in arrs]


def _conv_inputs(seed, L, r):
    K = L * (2 * r + 1) ** 3
    bound = 1.0 / np.sqrt(K)
    return prng.uniform(seed, (96, K), -bound, bound), prng.uniform(seed + 1, (96,), -bound, bound)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("case", PROJ_CASES)
def test_golden_reference(case, precision):
    import dvccorr
    g = load_golden(case + ".npz")
    f1, f2, coords, w, b, L, r, legacy = proj_inputs(g)
    t1, t2, tc, tw, tb = _gpu(f1, f2, coords, w, b)
    blk = dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision)
    out = blk.lookup_convc1(tc, tw, tb)
    torch.cuda.synchronize()
    assert out.shape == g["out"].shape and out.dtype == torch.float32
    assert orc.rel_err(out.cpu().numpy(), g["out"]) < (PROJ_TOL if precision == "bf16" else FP32_TOL)


@pytest.mark.parametrize("shape,C,L,r,legacy", [
    ((9, 7, 5), 32, 2, 1, False),      # ragged tile (315 queries), non-cubic
    ((12, 10, 16), 64, 3, 2, False),
    ((16, 16, 16), 32, 4, 3, False),   # level 3 = 2^3
    ((8, 8, 8), 16, 4, 4, True),       # level 3 = 1^3: zero level
    ((10, 12, 12), 32, 2, 4, True),    # legacy with W == D
    ((11, 9, 13), 32, 3, 4, False),
])
def test_against_oracle(shape, C, L, r, legacy):
    import dvccorr
    H, W, D = shape
    seed = 900 + H + 3 * W + 7 * D + r
    f1 = prng.normal(seed, (1, C, H, W, D))
    f2 = prng.normal(seed + 1, (1, C, H, W, D))
    coords = prng.flow_coords(seed + 2, 1, H, W, D, 2.5)
    w, b = _conv_inputs(seed + 3, L, r)
    ref = orc.motion_convc1(orc.corr_lookup(f1, f2, coords, L, r, legacy), w, b)
    t1, t2, tc, tw, tb = _gpu(f1, f2, coords, w, b)
    for precision in ("fp32", "bf16"):
        blk = dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision)
        out = blk.lookup_convc1(tc, tw, tb).cpu().numpy()
        assert orc.rel_err(out, ref) < (PROJ_TOL if precision == "bf16" else FP32_TOL), precision


def test_nonfinite_coords_give_relu_bias():
    """NaN / huge coordinates sample zeros (as grid_sample does), so convc1 sees 0 there: relu(b)."""
    import dvccorr
    H = W = D = 8
    f1 = prng.normal(31, (1, 16, H, W, D))
    f2 = prng.normal(32, (1, 16, H, W, D))
    coords = prng.flow_coords(33, 1, H, W, D, 1.0)
    coords[0, :, 1, 2, 3] = np.nan
    coords[0, 0, 4, 4, 4] = 1e30
    w, b = _conv_inputs(34, 2, 4)
    t1, t2, tc, tw, tb = _gpu(f1, f2, coords, w, b)
    out = dvccorr.CorrBlock(t1, t2, 2, 4, precision="bf16").lookup_convc1(tc, tw, tb).cpu().numpy()
    relu_b = np.maximum(b, 0).astype(np.float32)
    np.testing.assert_allclose(out[0, :, 1, 2, 3], relu_b, rtol=0, atol=1e-6)
    np.testing.assert_allclose(out[0, :, 4, 4, 4], relu_b, rtol=0, atol=1e-6)
    assert np.isfinite(out).all()


def test_bench_size_against_unfused_and_deterministic():
    """32^3 x 128, L=4, r=4 (the bench config): fused vs relu(conv3d(lookup)) on the GPU; bitwise repeatable."""
    import dvccorr
    S, C, L, r = 32, 128, 4, 4
    g = torch.Generator(device="cpu").manual_seed(77)
    f1 = torch.randn(1, C, S, S, S, generator=g).to(DEV)
    f2 = torch.randn(1, C, S, S, S, generator=g).to(DEV)
    base = dvccorr.coords_grid_3d(1, S, S, S, DEV)
    coords = base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2).to(DEV)
    w, b = (torch.from_numpy(a).to(DEV) for a in _conv_inputs(78, L, r))
    blk = dvccorr.CorrBlock(f1, f2, L, r, precision="bf16")
    ref = torch.relu(torch.nn.functional.conv3d(blk(coords), w.view(96, -1, 1, 1, 1), b))
    out = blk.lookup_convc1(coords, w, b)
    out2 = blk.lookup_convc1(coords, w, b)
    torch.cuda.synchronize()
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < FUSED_VS_UNFUSED_TOL, err     # same pyramid: only the fp16 operand rounding differs
    assert torch.equal(out, out2)


def test_unsupported_radius_falls_back_and_direct_call_raises():
    import dvccorr
    from dvccorr import ops
    H = W = D = 12
    f1 = prng.normal(41, (1, 16, H, W, D))
    f2 = prng.normal(42, (1, 16, H, W, D))
    coords = prng.flow_coords(43, 1, H, W, D, 1.0)
    w, b = _conv_inputs(44, 1, 5)
    t1, t2, tc, tw, tb = _gpu(f1, f2, coords, w, b)
    blk = dvccorr.CorrBlock(t1, t2, 1, 5, precision="fp32")
    out = blk.lookup_convc1(tc, tw, tb)       # r = 5: the unfused composition
    ref = orc.motion_convc1(orc.corr_lookup(f1, f2, coords, 1, 5, False), w, b)
    assert orc.rel_err(out.cpu().numpy(), ref) < 1e-5
    with pytest.raises(NotImplementedError):
        ops.proj_pack(tw, 1, 5, False)
    with pytest.raises(ValueError):
        ops.proj_pack(tw[:, :100], 1, 4, False)


def test_fp32_block_fused_exact_at_bench_size():
    """fp32 pyramid (the reference's fp32 evaluation, evaluate_phase1.py:115-131) at the bench shape: the fused
    exact consumer (dvc_proj_pack_exact + dvc_corr_lookup_proj, never the composition) against relu(conv3d(lookup))
    on the same pyramid at 1e-5, and bitwise repeatable."""
    import dvccorr
    S, C, L, r = 32, 128, 4, 4
    g = torch.Generator(device="cpu").manual_seed(79)
    f1 = torch.randn(1, C, S, S, S, generator=g).to(DEV)
    f2 = torch.randn(1, C, S, S, S, generator=g).to(DEV)
    base = dvccorr.coords_grid_3d(1, S, S, S, DEV)
    coords = base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2).to(DEV)
    w, b = (torch.from_numpy(a).to(DEV) for a in _conv_inputs(80, L, r))
    blk = dvccorr.CorrBlock(f1, f2, L, r, precision="fp32")
    ref = torch.relu(torch.nn.functional.conv3d(blk(coords), w.view(96, -1, 1, 1, 1), b))

    def _no_composition(*a, **k):
        raise AssertionError("fp32 lookup_convc1 took the composition")
    blk._convc1_composition = _no_composition
    out = blk.lookup_convc1(coords, w, b)
    out2 = blk.lookup_convc1(coords, w, b)
    torch.cuda.synchronize()
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < FP32_TOL, err
    assert torch.equal(out, out2)
