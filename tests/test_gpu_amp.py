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
    # fp16 inputs default to fp16, the on-the-fly block keeps bf16 operands
    assert dvccorr.CorrBlock(t1.half(), t2.half(), L, r).precision == "fp16"
    assert dvccorr.CorrBlockFused(t1, t2, L, r, precision="fp16").precision == "bf16"


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
    """Gradients of an fp16 block (fp32 VALU gradient kernels over fp16 operands) against autograd through the
    fp32 CPU restatement, at the AMP tolerance (the operands carry fp16 rounding)."""
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
