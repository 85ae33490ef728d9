"""GPU: the AMP (fp16) pyramid -- the reference's CorrBlock under its Trainer's autocast.

The reference Trainer runs the model under torch.amp.autocast('cuda')
(src/training/trainer.py:249-252), so CorrBlock's matmul and pyramid are float16
(src/core/corr.py:155-167) and the lookup output float32 (corr.py:208).
precision="fp16" (the default inside an enabled float16 autocast region) packs
fp16 operands, builds on v_mfma_f32_32x32x16_f16 and stores fp16.

Golden vectors: tests/golden/amp_*.npz, the reference CorrBlock run here under
torch.autocast('cpu', dtype=torch.float16) (tests/golden/gen_amp_golden.py; CPU
autocast pools level 0 in float32, CUDA in float16 -- one fp16 rounding apart).
Tolerance: max|out - ref| / max|ref| <= 5e-3, the reference's own fp16-autocast
bound (tests/test_corr_equivalence.py:156-186).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch

import prng
from conftest import GOLDEN, load_golden, oracle_grads, proj_inputs
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
AMP_TOL = 5e-3
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "amp_*.npz")))


def amp_case(name):
    g = load_golden(name + ".npz")
    B, C, H, W, D, L, r = (int(v) for v in g["shape"])
    seed = int(g["seed"][0])
    f1 = prng.normal(seed, (B, C, H, W, D))
    f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, float(g["max_flow"][0]))
    return g, f1, f2, coords, L, r, bool(int(g["legacy"][0]))


def _compare(out, g):
    if "out" in g:
        return orc.rel_err(out, g["out"])
    B, Ch = out.shape[:2]
    flat = out.reshape(B, Ch, -1)
    N = flat.shape[2]
    rows = np.stack([flat[q // N, :, q % N] for q in g["rows"]])
    return orc.rel_err(rows, g["out_rows"])


@pytest.mark.parametrize("build", ["gemm", "pool"])
@pytest.mark.parametrize("case", CASES)
def test_fp16_pyramid_against_reference_amp(case, build):
    import dvccorr
    g, f1, f2, coords, L, r, legacy = amp_case(case)
    t1, t2, tc = (torch.from_numpy(a).to(DEV) for a in (f1, f2, coords))
    with torch.no_grad():
        blk = dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision="fp16", build=build)
        out = blk(tc)
    assert blk.precision == "fp16" and out.dtype == torch.float32
    assert blk.corr_pyramid[0].dtype == torch.float16
    e = _compare(out.cpu().numpy(), g)
    assert e <= AMP_TOL, (case, build, e)


def test_autocast_default_is_fp16_and_closer_than_bf16():
    """Inside torch.amp.autocast('cuda') the block builds fp16 like the reference; that pyramid is closer
    to the reference's AMP output than a bf16 one (7 vs 10 mantissa bits)."""
    import dvccorr
    g, f1, f2, coords, L, r, legacy = amp_case("amp_888_L4_r4")
    t1, t2, tc = (torch.from_numpy(a).to(DEV) for a in (f1, f2, coords))
    with torch.no_grad():
        with torch.amp.autocast("cuda"):
            blk = dvccorr.CorrBlock(t1, t2, L, r)
            out = blk(tc)
        bf = dvccorr.CorrBlock(t1, t2, L, r, precision="bf16")(tc)
        with torch.amp.autocast("cuda", dtype=torch.bfloat16):
            assert dvccorr.CorrBlock(t1, t2, L, r).precision == "bf16"
    assert blk.precision == "fp16" and out.dtype == torch.float32
    e16, ebf = _compare(out.cpu().numpy(), g), _compare(bf.cpu().numpy(), g)
    assert e16 <= AMP_TOL and e16 < ebf, (e16, ebf)
    # fp16 inputs default to fp16; the on-the-fly block follows the same policy (round 4: fp16 MFMA operands,
    # as the reference's CorrBlockOnTheFly einsum under autocast, corr_otf.py:198-237)
    assert dvccorr.CorrBlock(t1.half(), t2.half(), L, r).precision == "fp16"
    assert dvccorr.CorrBlockFused(t1, t2, L, r, precision="fp16").precision == "fp16"
    with torch.amp.autocast("cuda"):
        assert dvccorr.CorrBlockFused(t1, t2, L, r).precision == "fp16"
        assert dvccorr.CorrBlockOnTheFly(t1, t2, L, r).precision == "fp16"


def test_fp16_bricked_equals_linear_and_walk():
    """The fp16 tile kernel reads bricked and linear pyramids to the same bits, and agrees bitwise with the
    lane-per-query walk (same arithmetic) -- config #3's shape (32^3, C = 128, L = 4, r = 4)."""
    import dvccorr
    from dvccorr import _lib
    S, C, L, r = 32, 128, 4, 4
    f1 = torch.from_numpy(prng.normal(31, (1, C, S, S, S))).to(DEV)
    f2 = torch.from_numpy(prng.normal(32, (1, C, S, S, S))).to(DEV)
    tc = torch.from_numpy(prng.flow_coords(33, 1, S, S, S, 2.0)).to(DEV)
    with torch.no_grad():
        a = dvccorr.CorrBlock(f1, f2, L, r, precision="fp16")(tc)
        lin = dvccorr.CorrBlock(f1, f2, L, r, precision="fp16", bricked=False)
        b = lin(tc)
        _lib.set_tuning("lookup_variant", 0)
        try:
            c = lin(tc)
        finally:
            _lib.set_tuning("lookup_variant", 2)
    assert torch.equal(a, b) and torch.equal(b, c)
    rows = np.arange(0, S ** 3, 997)
    ref = orc.corr_lookup(f1.cpu().numpy(), f2.cpu().numpy(), tc.cpu().numpy(), L, r, False, rows=rows)
    got = a.reshape(1, L * (2 * r + 1) ** 3, -1)[0][:, rows].T.cpu().numpy()
    assert orc.rel_err(got, ref) <= AMP_TOL


@pytest.mark.parametrize("name", ["proj_888_L2_r4", "proj_888_L2_r4_legacy", "proj_978_L3_r3"])
def test_fp16_convc1_fused(name):
    """convc1 fused into the fp16 block's lookup (dvc_corr_lookup_proj with fp16 pyramid rows), against the
    reference's CorrBlock + MotionEncoder.convc1 + ReLU (tests/golden/proj_*.npz) at the fused tolerance 1e-2."""
    import dvccorr
    g = load_golden(name + ".npz")
    f1, f2, coords, w, b, L, r, legacy = proj_inputs(g)
    t = lambda a: torch.from_numpy(a).to(DEV)
    with torch.no_grad():
        blk = dvccorr.CorrBlock(t(f1), t(f2), L, r, legacy_wd_swap=legacy, precision="fp16")
        out = blk.lookup_convc1(t(coords), t(w), t(b))
    assert orc.rel_err(out.cpu().numpy(), g["out"]) <= 1e-2


def test_fp16_backward():
    """Gradients of an fp16 block (round 4: the fp16 MFMA gradient kernels, window gradients as fp16 hi/lo pairs)
    against autograd through the fp32 CPU restatement, at the AMP tolerance (the operands carry fp16 rounding)."""
    import dvccorr
    H, W, D, C, L, r = 8, 12, 10, 32, 3, 3
    f1, f2 = prng.normal(801, (1, C, H, W, D)), prng.normal(802, (1, C, H, W, D))
    coords = prng.flow_coords(803, 1, H, W, D, 2.5)
    G = prng.normal(804, (1, L * (2 * r + 1) ** 3, H, W, D))
    ref1, ref2 = oracle_grads(f1, f2, coords, G, L, r, False)
    t1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    t2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    out = dvccorr.CorrBlock(t1, t2, L, r, precision="fp16")(torch.from_numpy(coords).to(DEV))
    (out * torch.from_numpy(G).to(DEV)).sum().backward()
    e1, e2 = orc.rel_err(t1.grad.cpu().numpy(), ref1), orc.rel_err(t2.grad.cpu().numpy(), ref2)
    assert e1 <= AMP_TOL and e2 <= AMP_TOL, (e1, e2)


# ---- the on-the-fly block in fp16 (round 4): the reference's CorrBlockOnTheFly under autocast runs its einsum in
# fp16 (corr_otf.py:198-237); k_fused_box / k_fused_proj take fp16 operands on v_mfma_f32_16x16x32_f16 and round
# the window dots to fp16 exactly as the fp16 build rounds its pyramid.


@pytest.mark.parametrize("shape,C,L,r", [((9, 7, 20), 32, 2, 4), ((16, 12, 40), 64, 3, 3), ((8, 8, 24), 128, 2, 2),
                                         ((12, 10, 17), 32, 2, 1)])
def test_fp16_fused_matches_materialised(shape, C, L, r):
    """The fp16 on-the-fly kernels reproduce the fp16 materialised pyramid + lookup bit for bit (box kernel
    variants 2, 3, 4; variant 1, the bf16-only tile kernel, falls back to the default box), ragged boxes, NaN /
    huge coordinates, both conventions (legacy W != D levels: per-output kernel, AMP tolerance)."""
    import dvccorr
    from dvccorr import _lib
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(H * 1000 + W * 10 + D + r + C + 16)
    f1 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    base = dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu"))
    c = base + (torch.rand(1, 3, H, W, D, generator=g) * 2 - 1) * (r + 4)
    c.view(3, -1)[:, 5] = float("nan")
    c.view(3, -1)[1, 17] = 1e30
    c = c.to(DEV)
    lay = dvccorr.layout(H, W, D, L, C)
    n3 = (2 * r + 1) ** 3
    with torch.no_grad():
        for legacy in (False, True):
            ref = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision="fp16")(c)
            fz = dvccorr.CorrBlockFused(f1, f2, L, r, legacy_wd_swap=legacy, precision="fp16")
            assert fz.precision == "fp16"
            try:
                _lib.set_tuning("fused_variant", 0)
                two_stage = fz(c)
                for variant in (1, 2, 3, 4):
                    _lib.set_tuning("fused_variant", variant)
                    out = fz(c)
                    assert torch.isfinite(out).all(), variant
                    for l, (h, w, d) in enumerate(lay.levels()):
                        sl = slice(l * n3, (l + 1) * n3)
                        if legacy and w != d and min(h, w, d) > 1:
                            assert orc.rel_err(out[:, sl].cpu().numpy(), ref[:, sl].cpu().numpy()) <= AMP_TOL
                        else:
                            assert torch.equal(out[:, sl], ref[:, sl]), (variant, shape, l, legacy)
                    assert orc.rel_err(out.cpu().numpy(), two_stage.cpu().numpy()) <= AMP_TOL, variant
            finally:
                _lib.set_tuning("fused_variant", 2)


@pytest.mark.parametrize("case", CASES)
def test_fp16_fused_against_reference_amp(case):
    """The on-the-fly block in fp16 against the reference's own AMP output (tests/golden/amp_*.npz) at 5e-3."""
    import dvccorr
    g, f1, f2, coords, L, r, legacy = amp_case(case)
    t1, t2, tc = (torch.from_numpy(a).to(DEV) for a in (f1, f2, coords))
    with torch.no_grad():
        with torch.amp.autocast("cuda"):
            blk = dvccorr.CorrBlockFused(t1, t2, L, r, legacy_wd_swap=legacy)
            out = blk(tc)
    assert blk.precision == "fp16" and out.dtype == torch.float32
    e = _compare(out.cpu().numpy(), g)
    assert e <= AMP_TOL, (case, e)


@pytest.mark.parametrize("name", ["proj_888_L2_r4", "proj_888_L2_r4_legacy", "proj_978_L3_r3", "proj_888_L4_r1"])
def test_fp16_fused_convc1(name):
    """convc1 fused into the fp16 on-the-fly lookup (k_fused_proj with fp16 dots): against the reference's
    CorrBlock + MotionEncoder.convc1 + ReLU (tests/golden/proj_*.npz) at 1e-2, and within 1e-5 of the fp16
    materialised block's fused convc1 (same dots, same fp16 X operands, sorted query order)."""
    import dvccorr
    g = load_golden(name + ".npz")
    f1, f2, coords, w, b, L, r, legacy = proj_inputs(g)
    t = lambda a: torch.from_numpy(a).to(DEV)
    with torch.no_grad():
        fz = dvccorr.CorrBlockFused(t(f1), t(f2), L, r, legacy_wd_swap=legacy, precision="fp16")
        out = fz.lookup_convc1(t(coords), t(w), t(b))
        mat = dvccorr.CorrBlock(t(f1), t(f2), L, r, legacy_wd_swap=legacy, precision="fp16").lookup_convc1(
            t(coords), t(w), t(b))
    assert orc.rel_err(out.cpu().numpy(), g["out"]) <= 1e-2
    assert orc.rel_err(out.cpu().numpy(), mat.cpu().numpy()) <= 1e-5


def test_fp16_fused_backward():
    """Gradients of the fp16 on-the-fly block (dvc_corr_backward over its fp16 packed operands, MFMA path)
    against autograd through the fp32 CPU restatement at the AMP tolerance."""
    import dvccorr
    H, W, D, C, L, r = 10, 8, 12, 64, 3, 4
    f1, f2 = prng.normal(811, (1, C, H, W, D)), prng.normal(812, (1, C, H, W, D))
    coords = prng.flow_coords(813, 1, H, W, D, 2.5)
    G = prng.normal(814, (1, L * (2 * r + 1) ** 3, H, W, D))
    ref1, ref2 = oracle_grads(f1, f2, coords, G, L, r, False)
    t1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    t2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    with torch.amp.autocast("cuda"):
        blk = dvccorr.CorrBlockFused(t1, t2, L, r)
        out = blk(torch.from_numpy(coords).to(DEV))
        loss = (out * torch.from_numpy(G).to(DEV)).sum()
    assert blk.precision == "fp16"
    loss.backward()
    e1, e2 = orc.rel_err(t1.grad.cpu().numpy(), ref1), orc.rel_err(t2.grad.cpu().numpy(), ref2)
    assert e1 <= AMP_TOL and e2 <= AMP_TOL, (e1, e2)
