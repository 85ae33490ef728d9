"""GPU parity: the HIP path (through the C ABI) against the golden vectors and
the CPU oracle.

Tolerances (north_star): max|out - ref| / max|ref|
  fp32 build + lookup     <= 1e-5
  bf16-MFMA build         <= 1e-2
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch

import prng
from conftest import GOLDEN, corr_inputs, load_golden
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

FP32_TOL = 1e-5
BF16_TOL = 1e-2
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "equiv_*.npz"))) + \
    sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "edge_*.npz")))

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _no_grad():
    with torch.no_grad():
        yield


def _gpu(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in arrs]


def _rows(out: torch.Tensor, rows) -> np.ndarray:
    B, Ch = out.shape[:2]
    flat = out.reshape(B, Ch, -1).cpu().numpy()
    N = flat.shape[2]
    return np.stack([flat[r // N, :, r % N] for r in rows])


def _blocks(kind, t1, t2, L, r, legacy, precision):
    import dvccorr
    if kind == "gemm":
        return dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision)
    if kind == "pool":
        return dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision, build="pool")
    return dvccorr.CorrBlockFused(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision)


@pytest.mark.parametrize("kind", ["gemm", "pool", "fused"])
@pytest.mark.parametrize("case", CASES)
def test_small_cases_fp32(case, kind):
    g = load_golden(case + ".npz")
    f1, f2, coords, L, r = corr_inputs(g)
    t1, t2, tc = _gpu(f1, f2, coords)
    for legacy, tag in ((False, "fixed"), (True, "legacy")):
        out = _blocks(kind, t1, t2, L, r, legacy, "fp32")(tc)
        assert out.shape == (f1.shape[0], L * (2 * r + 1) ** 3) + f1.shape[2:]
        assert out.dtype == torch.float32 and out.is_contiguous()
        e = orc.rel_err(_rows(out, g["rows"]), g[f"out_rows_{tag}"])
        assert e <= FP32_TOL, (case, kind, tag, e)
        full = orc.corr_lookup(f1, f2, coords, L, r, legacy)
        e = orc.rel_err(out.cpu().numpy(), full)
        assert e <= FP32_TOL, (case, kind, tag, "full", e)


@pytest.mark.parametrize("kind", ["gemm", "fused"])
@pytest.mark.parametrize("case", ["equiv_L4_r4", "edge_978_L3_r3", "cfg2"])
def test_bf16_build(case, kind):
    g = load_golden(case + ".npz")
    f1, f2, coords, L, r = corr_inputs(g)
    t1, t2, tc = _gpu(f1, f2, coords)
    for legacy, tag in ((False, "fixed"), (True, "legacy")):
        out = _blocks(kind, t1, t2, L, r, legacy, "bf16")(tc)
        e = orc.rel_err(_rows(out, g["rows"]), g[f"out_rows_{tag}"])
        assert e <= BF16_TOL, (case, kind, tag, e)


@pytest.mark.parametrize("kind", ["gemm", "pool", "fused"])
def test_cfg2_fp32_checksums(kind):
    """Config #2 (16^3, C=128, L=4, r=4) fp32: sampled rows + full-output checksums."""
    g = load_golden("cfg2.npz")
    f1, f2, coords, L, r = corr_inputs(g)
    t1, t2, tc = _gpu(f1, f2, coords)
    out = _blocks(kind, t1, t2, L, r, False, "fp32")(tc)
    assert orc.rel_err(_rows(out, g["rows"]), g["out_rows_fixed"]) <= FP32_TOL
    o = out.double()
    cs = g["checksum_fixed"]
    assert abs(o.abs().max().item() - cs[3]) / cs[3] < FP32_TOL
    assert abs((o * o).sum().item() - cs[2]) / cs[2] < 1e-6
    sums = o.reshape(1, L, -1).sum(-1)[0].cpu().numpy()
    np.testing.assert_allclose(sums, g["level_sums_fixed"], rtol=1e-4, atol=1e-3 * cs[3])


@pytest.mark.parametrize("precision,tol", [("fp32", FP32_TOL), ("bf16", BF16_TOL)])
def test_cfg3_rows(precision, tol):
    """Config #3 (32^3, C=128, L=4, r=4): the bench workload, sampled rows vs the reference."""
    import dvccorr
    g = load_golden("cfg3.npz")
    f1, f2, coords, L, r = corr_inputs(g)
    t1, t2, tc = _gpu(f1, f2, coords)
    blk = dvccorr.CorrBlock(t1, t2, L, r, precision=precision)
    out = blk(tc)
    for legacy, tag in ((False, "fixed"), (True, "legacy")):
        if legacy:
            blk.legacy_wd_swap = True
            out = blk(tc)
        e = orc.rel_err(_rows(out, g["rows"]), g[f"out_rows_{tag}"])
        assert e <= tol, (precision, tag, e)
    cs = g["checksum_fixed"]
    if precision == "fp32":
        blk.legacy_wd_swap = False
        o = blk(tc).double()
        assert abs((o * o).sum().item() - cs[2]) / cs[2] < 1e-5
    # pyramid rows through the reference-shaped zero-copy views
    pyr = blk.corr_pyramid
    assert [tuple(p.shape[2:]) for p in pyr] == [(32, 32, 32), (16, 16, 16), (8, 8, 8), (4, 4, 4)]
    prow = g["rows"][: g["pyr_rows"].shape[0]]
    got = np.concatenate([p.reshape(p.shape[0], -1)[torch.from_numpy(prow).to(DEV)].float().cpu().numpy()
                          for p in pyr], axis=1)
    assert orc.rel_err(got, g["pyr_rows"]) <= tol


def test_sampler_kats():
    import dvccorr
    g = load_golden("sampler_kat.npz")
    v = torch.zeros(1, 1, 8, 12, 16, device=DEV)
    v[0, 0, 3, 7, 11] = 1.0
    q = torch.from_numpy(g["imp_queries"]).to(DEV)
    np.testing.assert_array_equal(dvccorr.bilinear_sampler_3d(v, q).cpu().numpy(), g["imp_fixed"])
    np.testing.assert_array_equal(dvccorr.bilinear_sampler_3d(v, q, legacy_wd_swap=True).cpu().numpy(),
                                  g["imp_legacy"])
    cube = torch.zeros(1, 1, 16, 16, 16, device=DEV)
    cube[0, 0, 3, 7, 11] = 1.0
    cq = torch.from_numpy(g["cube_queries"]).to(DEV)
    np.testing.assert_array_equal(dvccorr.bilinear_sampler_3d(cube, cq, True).cpu().numpy(), g["cube_legacy"])
    rv = torch.from_numpy(prng.normal(101, (1, 2, 9, 7, 8))).to(DEV)
    pts = torch.from_numpy(g["rand_pts"]).to(DEV)
    for leg, key in ((False, "rand_fixed"), (True, "rand_legacy")):
        assert orc.rel_err(dvccorr.bilinear_sampler_3d(rv, pts, leg).cpu().numpy(), g[key]) <= 1e-6


def test_peak_location():
    """test_corr_sampler.py:74-105: the 9^3 window argmax sits at the true shift (fixed), drifts (legacy)."""
    import dvccorr
    g = load_golden("peak_shift.npz")
    G, C = int(g["G"][0]), int(g["C"][0])
    shift = tuple(int(s) for s in g["shift"])
    f2 = prng.normal(int(g["seed"][0]), (1, C, G, G, G))
    f1 = np.roll(f2, tuple(-s for s in shift), axis=(2, 3, 4)).copy()
    t1, t2 = _gpu(f1, f2)
    coords = dvccorr.coords_grid_3d(1, G, G, G, DEV)
    for legacy, key in ((False, "out_fixed"), (True, "out_legacy")):
        for kind in ("gemm", "fused"):
            out = _blocks(kind, t1, t2, 1, 4, legacy, "fp32")(coords)
            probes = np.stack([out[0, :, h, w, d].cpu().numpy() for (h, w, d) in g["probes"]])
            assert orc.rel_err(probes, g[key]) <= FP32_TOL
            offs = [tuple(int(i) - 4 for i in np.unravel_index(int(np.argmax(p)), (9, 9, 9))) for p in probes]
            assert (offs == [shift] * 4) != legacy


def test_zero_levels_and_errors():
    import dvccorr
    f = torch.randn(1, 8, 8, 8, 2, device=DEV)
    with pytest.raises(RuntimeError):
        dvccorr.CorrBlock(f, f, 3, 4)
    blk = dvccorr.CorrBlock(f, f, 2, 2)
    out = blk(dvccorr.coords_grid_3d(1, 8, 8, 2, DEV))
    assert out[:, 125:].abs().max().item() == 0.0      # level 1 is (4,4,1): all zeros (corr.py:41-44)
    assert out[:, :125].abs().max().item() > 0.0
    with pytest.raises(ValueError):
        blk(torch.zeros(1, 3, 8, 8, 3, device=DEV))


def test_nonfinite_coords_give_zero():
    """NaN / huge coordinates: every corner out of range in the reference -> 0 (no NaN leaks)."""
    import dvccorr
    f1 = torch.randn(1, 16, 8, 8, 8, device=DEV)
    f2 = torch.randn(1, 16, 8, 8, 8, device=DEV)
    c = dvccorr.coords_grid_3d(1, 8, 8, 8, DEV).clone()
    c[0, 0, 1, 2, 3] = float("nan")
    c[0, 1, 4, 4, 4] = 1e30
    c[0, 2, 5, 5, 5] = -1e9
    for kind in ("gemm", "fused"):
        out = _blocks(kind, f1, f2, 2, 4, False, "fp32")(c)
        assert torch.isfinite(out).all()
        for (h, w, d) in ((1, 2, 3), (4, 4, 4), (5, 5, 5)):
            assert out[0, :, h, w, d].abs().max().item() == 0.0
        ref = orc.corr_lookup(f1.cpu().numpy(), f2.cpu().numpy(), c.cpu().numpy(), 2, 4, False)
        assert orc.rel_err(out.cpu().numpy(), ref) <= FP32_TOL


def test_plumbing_iterations():
    """Config #1: the fmaps and per-iteration coords RAFTDVC fed the reference CorrBlock (64^3, 1/8, L=4)."""
    import dvccorr
    g = load_golden("plumbing.npz")
    t1, t2 = _gpu(g["fmap1"], g["fmap2"])
    for kind in ("gemm", "fused"):
        blk = _blocks(kind, t1, t2, 4, 4, False, "fp32")
        for it in range(g["coords"].shape[0]):
            out = blk(_gpu(g["coords"][it])[0])
            assert orc.rel_err(_rows(out, g["rows"]), g["out_rows"][it]) <= FP32_TOL, (kind, it)
            cs = g["out_checksums"][it]
            o = out.double()
            assert abs((o * o).sum().item() - cs[2]) / cs[2] < 1e-5
    # the reference-signature on-the-fly block is legacy-only, like corr_otf.py
    otf = dvccorr.CorrBlockOnTheFly(t1, t2, 4, 4)
    c0 = _gpu(g["coords"][0])[0]
    ref_leg = dvccorr.CorrBlock(t1, t2, 4, 4, legacy_wd_swap=True)(c0)
    assert orc.rel_err(otf(c0).cpu().numpy(), ref_leg.cpu().numpy()) <= FP32_TOL


def test_determinism_and_linearity_at_cfg3():
    """Size-independent properties at the bench size (bf16): bitwise determinism,
    exact scaling by 2 (power-of-two scale commutes with every rounding)."""
    import dvccorr
    S = 32
    f1 = torch.randn(1, 128, S, S, S, device=DEV)
    f2 = torch.randn(1, 128, S, S, S, device=DEV)
    c = torch.from_numpy(prng.flow_coords(77, 1, S, S, S, 2.0)).to(DEV)
    blk = dvccorr.CorrBlock(f1, f2, 4, 4, precision="bf16")
    a = blk(c)
    b = blk(c)
    assert torch.equal(a, b)
    blk2 = dvccorr.CorrBlock(f1 * 2, f2, 4, 4, precision="bf16")
    assert torch.equal(blk2(c), 2 * a)
    # the fused path agrees with the materialised one at the bench size
    fz = dvccorr.CorrBlockFused(f1, f2, 4, 4, precision="bf16")(c)
    assert orc.rel_err(fz.cpu().numpy(), a.cpu().numpy()) <= BF16_TOL


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_lookup_variants(variant):
    """Every lookup kernel (lane-per-query walk with unaligned runs / aligned chunks + v_perm, and the
    LDS-staged tile kernel) reproduces the golden rows."""
    import dvccorr
    from dvccorr import _lib
    _lib.set_tuning("lookup_variant", variant)
    try:
        for case, prec, tol in (("edge_978_L3_r3", "fp32", FP32_TOL), ("edge_965_L2_r4", "fp32", FP32_TOL),
                                ("cfg2", "fp32", FP32_TOL), ("cfg2", "bf16", BF16_TOL)):
            g = load_golden(case + ".npz")
            f1, f2, coords, L, r = corr_inputs(g)
            t1, t2, tc = _gpu(f1, f2, coords)
            for legacy, tag in ((False, "fixed"), (True, "legacy")):
                out = dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision=prec)(tc)
                e = orc.rel_err(_rows(out, g["rows"]), g[f"out_rows_{tag}"])
                assert e <= tol, (variant, case, prec, tag, e)
    finally:
        _lib.set_tuning("lookup_variant", 2)


@pytest.mark.parametrize("shape,L,r", [((9, 7, 5), 2, 1), ((12, 10, 16), 3, 2), ((16, 16, 16), 4, 3),
                                       ((20, 13, 24), 3, 4), ((32, 32, 32), 4, 4), ((24, 26, 28), 2, 5),
                                       ((30, 28, 40), 2, 6), ((40, 36, 33), 3, 4), ((16, 12, 20), 4, 4)])
def test_tile_kernel_matches_walk(shape, L, r):
    """The LDS-staged tile kernel (variant 2) is bit-identical to the lane-per-query walk (variant 0):
    same per-axis weights, same separable summation order; on the default block (wide levels in
    DVC_BRICKED bricks where the shape allows: the 32^3 case) and on a linear one.  Ragged tiles (Nq % 64 != 0), non-cubic and
    odd sizes, D padding, every radius the kernel is instantiated for, both conventions, both store
    dtypes, wide flows that leave the volume, and NaN / huge coordinates."""
    import dvccorr
    from dvccorr import _lib
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(H * 1000 + W * 10 + D + r)
    f1 = torch.randn(1, 32, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(1, 32, H, W, D, generator=g).to(DEV)
    base = dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu"))
    c = base + (torch.rand(1, 3, H, W, D, generator=g) * 2 - 1) * (r + 6)
    c.view(3, -1)[:, 5] = float("nan")
    c.view(3, -1)[1, 17] = 1e30
    c.view(3, -1)[2, 23] = -float("inf")
    c = c.to(DEV)
    try:
        for prec in ("bf16", "fp32"):
            for legacy in (False, True):
                # the walk reads the linear layout; the default block may store wide levels in bricks
                lin = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision=prec, bricked=False)
                blk = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision=prec)
                outs = []
                for v, b in ((0, lin), (2, blk)):
                    _lib.set_tuning("lookup_variant", v)
                    outs.append(b(c))
                _lib.set_tuning("lookup_variant", 2)
                outs.append(lin(c))   # the tile kernel on the linear layout too
                if r == 4:   # three 3-column waves (lookup_waves 0) vs the default four balanced waves
                    _lib.set_tuning("lookup_waves", 0)
                    outs.append(blk(c))
                    _lib.set_tuning("lookup_waves", 4)
                torch.cuda.synchronize()
                for k, o in enumerate(outs[2:]):
                    assert torch.equal(outs[0], o), (shape, L, r, prec, legacy, ("tile, linear", "lookup_waves 0")[k])
                assert torch.isfinite(outs[1]).all(), (prec, legacy)
                assert torch.equal(outs[0], outs[1]), (shape, L, r, prec, legacy,
                                                        float((outs[0] - outs[1]).abs().max()))
    finally:
        _lib.set_tuning("lookup_variant", 2)
        _lib.set_tuning("lookup_waves", 4)


@pytest.mark.parametrize("shape,C,L,r", [((9, 7, 5), 32, 2, 1), ((12, 10, 16), 64, 3, 2), ((16, 16, 16), 32, 4, 3),
                                         ((20, 13, 24), 128, 3, 4), ((32, 32, 32), 128, 4, 4),
                                         ((18, 34, 40), 64, 2, 4), ((8, 8, 8), 128, 2, 3)])
def test_fused_tile_matches_materialised(shape, C, L, r):
    """The MFMA fused kernels (no volume) reproduce the bf16 materialised pyramid + lookup bit for bit:
    k_fused_tile (variant 1: 2x2x16 query boxes, v_mfma_f32_32x32x16_bf16) and k_fused_cube (variants 2 and
    3: 4x4x4 query cubes, v_mfma_f32_16x16x32_bf16, 4 or 8 waves) -- the same scale-then-round to bf16 and
    the same interpolation arithmetic.  Ragged query boxes, non-cubic sizes, flows wide enough to push the
    union window past one MFMA z block, NaN / huge coordinates, both conventions.  Legacy levels with
    W != D go to the per-output kernel (fp32 dots of the same operands) and are held to BF16_TOL."""
    import dvccorr
    from dvccorr import _lib
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(H * 1000 + W * 10 + D + r + C)
    f1 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    base = dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu"))
    c = base + (torch.rand(1, 3, H, W, D, generator=g) * 2 - 1) * (r + 6)
    c.view(3, -1)[:, 5] = float("nan")
    c.view(3, -1)[1, 17] = 1e30
    c.view(3, -1)[2, 23] = -float("inf")
    c = c.to(DEV)
    lay = dvccorr.layout(H, W, D, L, C)
    n3 = (2 * r + 1) ** 3
    for legacy in (False, True):
        ref = dvccorr.CorrBlock(f1, f2, L, r, legacy_wd_swap=legacy, precision="bf16")(c)
        fz = dvccorr.CorrBlockFused(f1, f2, L, r, legacy_wd_swap=legacy, precision="bf16")
        try:
            _lib.set_tuning("fused_variant", 0)
            two_stage = fz(c)
            for variant in (1, 2, 3, 4):
                _lib.set_tuning("fused_variant", variant)
                out = fz(c)
                torch.cuda.synchronize()
                assert torch.isfinite(out).all(), variant
                for l, (h, w, d) in enumerate(lay.levels()):
                    sl = slice(l * n3, (l + 1) * n3)
                    if legacy and w != d and min(h, w, d) > 1:
                        e = orc.rel_err(out[:, sl].cpu().numpy(), ref[:, sl].cpu().numpy())
                        assert e <= BF16_TOL, (variant, shape, l, legacy, e)
                    else:
                        assert torch.equal(out[:, sl], ref[:, sl]), (variant, shape, C, L, r, l, legacy,
                                                                     float((out[:, sl] - ref[:, sl]).abs().max()))
                assert orc.rel_err(out.cpu().numpy(), two_stage.cpu().numpy()) <= BF16_TOL, variant
        finally:
            _lib.set_tuning("fused_variant", 2)


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
def test_fused_smooth_flow_bitwise(variant):
    """Bench-like inputs (identity + U(-2, 2) flow, 32^3 x 128, L=4, r=4): every fused MFMA variant equals
    the materialised bf16 path bit for bit over the whole output."""
    import dvccorr
    from dvccorr import _lib
    S, C, L, r = 32, 128, 4, 4
    g = torch.Generator(device="cpu").manual_seed(77)
    f1 = torch.randn(1, C, S, S, S, generator=g).to(DEV)
    f2 = torch.randn(1, C, S, S, S, generator=g).to(DEV)
    c = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) +
         (torch.rand(1, 3, S, S, S, generator=g) * 2 - 1) * 2).to(DEV)
    ref = dvccorr.CorrBlock(f1, f2, L, r, precision="bf16")(c)
    try:
        _lib.set_tuning("fused_variant", variant)
        out = dvccorr.CorrBlockFused(f1, f2, L, r, precision="bf16")(c)
    finally:
        _lib.set_tuning("fused_variant", 2)
    assert torch.equal(out, ref), float((out - ref).abs().max())


def test_fused_tile_slab():
    """The tile kernel on one rank's H-slab of queries (Nq = slab planes x W x D) equals the slab of the
    whole-grid result (the sharded layout of SURVEY 8(e))."""
    import dvccorr
    from dvccorr import ops
    H, W, D, C, L, r = 24, 20, 18, 64, 3, 4
    g = torch.Generator(device="cpu").manual_seed(5)
    f1 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(1, C, H, W, D, generator=g).to(DEV)
    c = (dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu")) +
         (torch.rand(1, 3, H, W, D, generator=g) * 2 - 1) * 3).to(DEV)
    dt = ops.dtype_code("bf16")
    t = ops.pack_targets(f2, L, dt)
    full = ops.lookup_fused(ops.pack_queries(f1.reshape(1, C, -1), dt), t, c.reshape(1, 3, -1), C, H, W, D, L, r,
                            False, dt)
    h0, h1 = 7, 15
    q = ops.pack_queries(f1[:, :, h0:h1].reshape(1, C, -1), dt)
    part = ops.lookup_fused(q, t, c[:, :, h0:h1].reshape(1, 3, -1), C, H, W, D, L, r, False, dt)
    assert torch.equal(part, full.view(1, -1, H, W, D)[:, :, h0:h1].reshape(1, -1, (h1 - h0) * W * D))


def test_graph_captured_iteration_loop():
    """The 12 GRU-iteration lookups + flow tails captured once in a HIP graph
    (torch.cuda.CUDAGraph over the C ABI: stream-ordered, allocation-free launches)
    and replayed on new coordinates give the eager results bit for bit."""
    import dvccorr
    S, C, L, r, iters = 16, 64, 4, 4, 12
    f1 = torch.from_numpy(prng.normal(900, (1, C, S, S, S))).to(DEV)
    f2 = torch.from_numpy(prng.normal(901, (1, C, S, S, S))).to(DEV)
    blk = dvccorr.CorrBlock(f1, f2, L, r, precision="bf16")
    deltas = [torch.from_numpy(prng.uniform(910 + i, (1, 3, S, S, S), -0.5, 0.5)).to(DEV) for i in range(iters)]
    c_static = torch.from_numpy(prng.flow_coords(902, 1, S, S, S, 2.0)).to(DEV)

    def loop(c):
        outs = []
        for i in range(iters):
            outs.append(blk(c))
            c, up = dvccorr.flow_step(c, deltas[i], (4 * S, 4 * S, 4 * S))
        return outs, c, up

    with torch.no_grad():
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            loop(c_static)   # warm-up outside capture
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            g_outs, g_c, g_up = loop(c_static)
        new_c = torch.from_numpy(prng.flow_coords(903, 1, S, S, S, 3.0)).to(DEV)
        c_static.copy_(new_c)
        g.replay()
        torch.cuda.synchronize()
        e_outs, e_c, e_up = loop(new_c)
        torch.cuda.synchronize()
    for a, b in zip(g_outs, e_outs):
        assert torch.equal(a, b)
    assert torch.equal(g_c, e_c) and torch.equal(g_up, e_up)
