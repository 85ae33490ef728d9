"""CPU: pin the oracle (oracle/) against the reference's golden vectors.

The golden vectors were produced by importing the reference
(tests/golden/gen_golden.py); here the oracle must reproduce them without
the reference.  Tolerance: max|oracle - ref| / max|ref| <= 2e-6 (the oracle
is float64, the reference float32), and exact for the KAT values.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest

import prng
from conftest import GOLDEN, corr_inputs, load_golden
from oracle import oracle as orc
from oracle import torch_cpu

CORR_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "equiv_*.npz"))) + \
    sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "edge_*.npz"))) + ["cfg2"]


def test_sampler_kat():
    g = load_golden("sampler_kat.npz")
    v = np.zeros((1, 1, 8, 12, 16), np.float32)
    v[0, 0, 3, 7, 11] = 1.0
    assert np.array_equal(orc.sample(v, g["imp_queries"], False).astype(np.float32), g["imp_fixed"])
    assert np.array_equal(orc.sample(v, g["imp_queries"], True).astype(np.float32), g["imp_legacy"])
    # reference KATs (test_corr_sampler.py:45-56): exact hit, transposed miss, 0.75 / 0.5 weights
    fixed = g["imp_fixed"].reshape(-1)
    assert fixed[0] == 1.0 and fixed[1] == 0.0 and fixed[2] == 0.0
    assert abs(fixed[3] - 0.75) < 1e-6 and abs(fixed[4] - 0.5) < 1e-6
    cube = np.zeros((1, 1, 16, 16, 16), np.float32)
    cube[0, 0, 3, 7, 11] = 1.0
    cl = orc.sample(cube, g["cube_queries"], True).reshape(-1)
    assert cl[0] == 0.0 and abs(cl[1] - 1.0) < 1e-6 and np.array_equal(cl.astype(np.float32), g["cube_legacy"].reshape(-1))
    rv = prng.normal(101, (1, 2, 9, 7, 8))
    for leg, key in ((False, "rand_fixed"), (True, "rand_legacy")):
        assert orc.rel_err(orc.sample(rv, g["rand_pts"], leg), g[key]) < 1e-6


def test_peak_shift():
    g = load_golden("peak_shift.npz")
    G, C = int(g["G"][0]), int(g["C"][0])
    shift = tuple(int(s) for s in g["shift"])
    f2 = prng.normal(int(g["seed"][0]), (1, C, G, G, G))
    f1 = np.roll(f2, tuple(-s for s in shift), axis=(2, 3, 4)).copy()
    coords = prng.identity_coords(1, G, G, G)
    N = G ** 3
    rows = np.array([(h * G + w) * G + d for (h, w, d) in g["probes"]], np.int64)
    for leg, key in ((False, "out_fixed"), (True, "out_legacy")):
        got = orc.corr_lookup(f1, f2, coords, 1, 4, leg, rows=rows)
        assert orc.rel_err(got, g[key]) < 2e-6
        offs = [tuple(int(i) - 4 for i in np.unravel_index(int(np.argmax(o)), (9, 9, 9))) for o in got]
        if not leg:
            assert offs == [shift] * 4
        else:
            assert offs != [shift] * 4
    assert N == 4096


@pytest.mark.parametrize("case", CORR_CASES)
def test_corr_case(case):
    g = load_golden(case + ".npz")
    f1, f2, coords, L, r = corr_inputs(g)
    rows = g["rows"]
    for leg, tag in ((False, "fixed"), (True, "legacy")):
        got = orc.corr_lookup(f1, f2, coords, L, r, leg, rows=rows)
        assert orc.rel_err(got, g[f"out_rows_{tag}"]) < 2e-6, (case, tag)
    pyr = orc.corr_rows(f1, f2, L, rows[: g["pyr_rows"].shape[0]])
    assert orc.rel_err(pyr, g["pyr_rows"]) < 2e-6


def test_cfg2_full_checksums():
    """Full 16^3 output from the oracle matches the reference's checksums."""
    g = load_golden("cfg2.npz")
    f1, f2, coords, L, r = corr_inputs(g)
    out = orc.corr_lookup(f1, f2, coords, L, r, False)
    cs = g["checksum_fixed"]
    assert abs(np.abs(out).max() - cs[3]) / cs[3] < 2e-6
    assert abs((out * out).sum() - cs[2]) / cs[2] < 2e-6
    assert abs(np.abs(out).sum() - cs[1]) / cs[1] < 2e-6


def test_torch_cpu_restatement_matches_golden():
    """The CPU-baseline restatement reproduces the reference rows bit-for-bit."""
    import torch
    g = load_golden("equiv_L2_r4.npz")
    f1, f2, coords, L, r = corr_inputs(g)
    for leg, tag in ((False, "fixed"), (True, "legacy")):
        out = torch_cpu.corr_lookup(torch.from_numpy(f1), torch.from_numpy(f2), torch.from_numpy(coords),
                                    L, r, leg).numpy()
        B, Ch = out.shape[:2]
        flat = out.reshape(B, Ch, -1)
        N = flat.shape[2]
        got = np.stack([flat[q // N, :, q % N] for q in g["rows"]])
        np.testing.assert_array_equal(got, g[f"out_rows_{tag}"])


GRAD_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "grad_*.npz")))


@pytest.mark.parametrize("case", GRAD_CASES)
def test_backward_oracle_matches_reference_gradients(case):
    """The backward oracle (autograd through oracle/torch_cpu.py) reproduces the gradients the reference's own
    autograd produced (tests/golden/gen_grad_golden.py; bitwise there, 1e-6 here to allow another BLAS)."""
    from conftest import grad_inputs, oracle_grads
    g = load_golden(case + ".npz")
    f1, f2, coords, G, L, r, legacy = grad_inputs(g)
    d1, d2 = oracle_grads(f1, f2, coords, G, L, r, legacy)
    if "grad_f1" in g:
        assert orc.rel_err(d1, g["grad_f1"]) < 1e-6 and orc.rel_err(d2, g["grad_f2"]) < 1e-6
    else:
        idx = g["idx"]
        assert orc.rel_err(d1.reshape(-1)[idx], g["grad_f1_s"]) < 1e-6
        assert orc.rel_err(d2.reshape(-1)[idx], g["grad_f2_s"]) < 1e-6
    for d, cs in ((d1, g["checksum_f1"]), (d2, g["checksum_f2"])):
        dd = d.astype(np.float64)
        assert abs((dd * dd).sum() - cs[2]) / cs[2] < 1e-6


def test_size1_level_raises_where_reference_raises():
    with pytest.raises(RuntimeError):
        orc.level_dims(8, 8, 2, 3)
    assert orc.level_dims(8, 8, 2, 2)[1] == (4, 4, 1)


def test_plumbing_fixture_consistent():
    """Config #1 capture: oracle reproduces every GRU iteration's sampled lookup rows."""
    g = load_golden("plumbing.npz")
    for it in (0, 5, 11):
        got = orc.corr_lookup(g["fmap1"], g["fmap2"], g["coords"][it], 4, 4, False, rows=g["rows"])
        assert orc.rel_err(got, g["out_rows"][it]) < 2e-6


PROJ_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "proj_*.npz")))


@pytest.mark.parametrize("case", PROJ_CASES)
def test_convc1_oracle_matches_reference(case):
    """oracle lookup + motion_convc1 against the reference's CorrBlock + MotionEncoder.convc1 + ReLU
    (tests/golden/gen_proj_golden.py): pins the channel order of the fused projection."""
    from conftest import proj_inputs
    g = load_golden(case + ".npz")
    f1, f2, coords, w, b, L, r, legacy = proj_inputs(g)
    ref = orc.motion_convc1(orc.corr_lookup(f1, f2, coords, L, r, legacy), w, b)
    assert orc.rel_err(ref, g["out"]) < 1e-5


AMP_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "amp_*.npz")))


@pytest.mark.parametrize("case", AMP_CASES)
def test_amp_fixture_reproduced_by_restatement(case):
    """The AMP (fp16) golden vectors (tests/golden/gen_amp_golden.py: the reference CorrBlock under
    torch.autocast('cpu', dtype=torch.float16)) are reproduced bit for bit by oracle/torch_cpu.py under the same
    autocast -- the restatement follows the reference's op sequence, so the fixtures are pinned here too."""
    import torch
    import prng
    from oracle import torch_cpu
    g = load_golden(case + ".npz")
    B, C, H, W, D, L, r = (int(v) for v in g["shape"])
    seed = int(g["seed"][0])
    f1 = prng.normal(seed, (B, C, H, W, D))
    f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, float(g["max_flow"][0]))
    legacy = bool(int(g["legacy"][0]))
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.float16):
        if "out" in g:
            out = torch_cpu.corr_lookup(torch.from_numpy(f1), torch.from_numpy(f2), torch.from_numpy(coords), L, r,
                                        legacy).float().numpy()
            assert np.array_equal(out, g["out"])
        else:   # sampled rows of the big case: per-row build + lookup over those rows
            rows = g["rows"]
            pyr = torch_cpu.build_rows(torch.from_numpy(f1), torch.from_numpy(f2), L, 0, B * H * W * D)
            out = torch_cpu.lookup_rows(pyr, torch.from_numpy(coords), r, legacy, 0, B * H * W * D).float().numpy()
            flat = out.reshape(B, out.shape[1], -1) if out.ndim > 2 else out
            got = np.stack([flat[q // (H * W * D), :, q % (H * W * D)] for q in rows])
            assert orc.rel_err(got, g["out_rows"]) < 1e-6
