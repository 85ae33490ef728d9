"""GPU: gradients of the correlation block w.r.t. both feature maps.

The reference trains through autograd of src/core/corr.py (matmul / avg_pool3d /
grid_sample); its own gradient check is tests/test_corr_equivalence.py:189-217.
Here dvc_corr_backward (raft-dvc_amd/csrc/backward.hip) is checked against the
gradients the reference itself produced (tests/golden/grad_*.npz, written by
tests/golden/gen_grad_golden.py) and against autograd through the CPU
restatement (oracle/torch_cpu.py, bit-identical to the reference on every golden
case) on further shapes, radii and conventions.

Tolerance: max|grad - ref| / max|ref| <= 1e-5 for the fp32 build (the kernels sum
in their own fixed order, ATen in its), <= 1e-2 for the bf16 build.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch

import prng
from conftest import GOLDEN, grad_inputs, load_golden, oracle_grads
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
GRAD_TOL = 1e-5
BF16_TOL = 1e-2
FP16_TOL = 5e-3     # the reference's AMP tolerance, test_corr_equivalence.py:156-186
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "grad_*.npz")))


def _gpu_grads(kind, f1, f2, coords, G, L, r, legacy, precision="fp32"):
    import dvccorr
    t1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    t2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    cls = dvccorr.CorrBlock if kind == "gemm" else dvccorr.CorrBlockFused
    out = cls(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision)(torch.from_numpy(coords).to(DEV))
    (out * torch.from_numpy(G).to(DEV)).sum().backward()
    return t1.grad.cpu().numpy(), t2.grad.cpu().numpy()


@pytest.mark.parametrize("kind", ["gemm", "fused"])
@pytest.mark.parametrize("case", CASES)
def test_grad_golden(case, kind):
    _check_golden(case, kind, "fp32", GRAD_TOL)


# The matrix-core gradient kernels (bf16 and, for the materialised block, fp16 operands) against the reference's
# own gradients at the production channel count and pyramid depth: grad_cfg2 is config #2's 16^3, C = 128, L = 4,
# r = 4 (the shapes k_grad_q_mfma / k_grad_t_mfma are benchmarked at, with more than one split per level).
@pytest.mark.parametrize("kind", ["gemm", "fused"])
@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp16", FP16_TOL)])
@pytest.mark.parametrize("case", ["grad_cfg2", "grad_edge_888_L4_r4", "grad_legacy_cube_L3_r2", "grad_equiv_L2_r4_rand"])
def test_grad_golden_low_precision(case, kind, precision, tol):
    _check_golden(case, kind, precision, tol)


@pytest.mark.parametrize("legacy", [False, True])
def test_grad_batch2_matrix_cores(legacy):
    """Batch 2 through the bf16 / fp16 MFMA gradient kernels (every (batch, level) pair is its own GEMM / window
    set): ragged 12 x 10 x 16 volumes, C = 128, L = 3, r = 4, flows that leave the volume, a different G per item."""
    B, (H, W, D), C, L, r = 2, (12, 10, 16), 128, 3, 4
    seed = 9100 + int(legacy)
    f1 = prng.normal(seed, (B, C, H, W, D))
    f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, r + 3.0)
    G = prng.normal(seed + 3, (B, L * (2 * r + 1) ** 3, H, W, D))
    ref1, ref2 = oracle_grads(f1, f2, coords, G, L, r, legacy)
    for precision, tol in (("bf16", BF16_TOL), ("fp16", FP16_TOL)):
        for kind in ("gemm", "fused"):
            d1, d2 = _gpu_grads(kind, f1, f2, coords, G, L, r, legacy, precision=precision)
            for b in range(B):   # per item, so a batch-offset bug cannot hide behind the other item's scale
                e1, e2 = orc.rel_err(d1[b], ref1[b]), orc.rel_err(d2[b], ref2[b])
                assert e1 <= tol and e2 <= tol, (kind, precision, legacy, b, e1, e2)


def _check_golden(case, kind, precision, tol):
    g = load_golden(case + ".npz")
    f1, f2, coords, G, L, r, legacy = grad_inputs(g)
    d1, d2 = _gpu_grads(kind, f1, f2, coords, G, L, r, legacy, precision=precision)
    assert np.isfinite(d1).all() and np.isfinite(d2).all()
    if "grad_f1" in g:
        e1, e2 = orc.rel_err(d1, g["grad_f1"]), orc.rel_err(d2, g["grad_f2"])
    else:
        idx = g["idx"]
        e1 = orc.rel_err(d1.reshape(-1)[idx], g["grad_f1_s"])
        e2 = orc.rel_err(d2.reshape(-1)[idx], g["grad_f2_s"])
        for d, cs in ((d1, g["checksum_f1"]), (d2, g["checksum_f2"])):
            dd = d.astype(np.float64)
            assert abs((dd * dd).sum() - cs[2]) / cs[2] < tol
    assert e1 <= tol and e2 <= tol, (case, kind, precision, e1, e2)


@pytest.mark.parametrize("shape,C,L,r,legacy", [((9, 7, 5), 32, 2, 1, False), ((12, 10, 16), 64, 3, 2, False),
                                                 ((16, 16, 16), 32, 4, 3, True), ((20, 13, 24), 128, 3, 4, False),
                                                 ((10, 12, 12), 32, 2, 5, True), ((14, 14, 14), 32, 2, 6, False)])
def test_grad_matches_oracle(shape, C, L, r, legacy):
    """Every instantiated radius, both conventions, ragged 4x4x4 boxes and bricks, flows that leave the volume
    (r + 3 voxels), against autograd through oracle/torch_cpu.py."""
    H, W, D = shape
    seed = H * 100 + W * 10 + D + r
    f1 = prng.normal(seed, (1, C, H, W, D))
    f2 = prng.normal(seed + 1, (1, C, H, W, D))
    coords = prng.flow_coords(seed + 2, 1, H, W, D, r + 3.0)
    G = prng.normal(seed + 3, (1, L * (2 * r + 1) ** 3, H, W, D))
    ref1, ref2 = oracle_grads(f1, f2, coords, G, L, r, legacy)
    for kind in ("gemm", "fused"):
        d1, d2 = _gpu_grads(kind, f1, f2, coords, G, L, r, legacy)
        e1, e2 = orc.rel_err(d1, ref1), orc.rel_err(d2, ref2)
        assert e1 <= GRAD_TOL and e2 <= GRAD_TOL, (shape, r, legacy, kind, e1, e2)


@pytest.mark.parametrize("precision,tol", [("fp32", GRAD_TOL), ("bf16", BF16_TOL)])
def test_grad_wide_features_c256(precision, tol):
    """C = 256 (C_pad 256, two 128-channel groups per gradient kernel; the reference's CUDA backward is
    templated for C in {16, 64, 128, 256}, corr_otf_cuda.cu:537-541) and C = 160 (a partial second group),
    against autograd through oracle/torch_cpu.py; tolerance test_corr_equivalence.py:189-217 style."""
    for C, shape, L, r in ((256, (10, 9, 12), 3, 4), (160, (8, 12, 10), 2, 3)):
        H, W, D = shape
        seed = 2560 + C + r
        f1 = prng.normal(seed, (1, C, H, W, D))
        f2 = prng.normal(seed + 1, (1, C, H, W, D))
        coords = prng.flow_coords(seed + 2, 1, H, W, D, 3.0)
        G = prng.normal(seed + 3, (1, L * (2 * r + 1) ** 3, H, W, D))
        ref1, ref2 = oracle_grads(f1, f2, coords, G, L, r, False)
        for kind in ("gemm", "fused"):
            d1, d2 = _gpu_grads(kind, f1, f2, coords, G, L, r, False, precision=precision)
            e1, e2 = orc.rel_err(d1, ref1), orc.rel_err(d2, ref2)
            assert e1 <= tol and e2 <= tol, (C, precision, kind, e1, e2)


def test_grad_bf16_build():
    g = load_golden("grad_equiv_L2_r4_rand.npz")
    f1, f2, coords, G, L, r, legacy = grad_inputs(g)
    for kind in ("gemm", "fused"):
        d1, d2 = _gpu_grads(kind, f1, f2, coords, G, L, r, legacy, precision="bf16")
        e1, e2 = orc.rel_err(d1, g["grad_f1"]), orc.rel_err(d2, g["grad_f2"])
        assert e1 <= BF16_TOL and e2 <= BF16_TOL, (kind, e1, e2)


def test_amp_policy_forward_and_grads():
    """AMP dtype policy: under torch.amp.autocast('cuda') (the reference Trainer,
    trainer.py:249-252) float32 fmaps (raft_dvc.py:366-367) build a 16-bit pyramid (fp16, as the reference's),
    lookups come back float32 and gradients reach both fmaps in float32; values within
    the bf16 tolerance of the reference's float32 outputs and gradients."""
    import dvccorr
    g = load_golden("grad_equiv_L2_r4_rand.npz")
    f1, f2, coords, G, L, r, legacy = grad_inputs(g)
    ref = orc.corr_lookup(f1, f2, coords, L, r, legacy)
    for cls in (dvccorr.CorrBlock, dvccorr.CorrBlockFused):
        t1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
        t2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
        with torch.amp.autocast("cuda"):
            blk = cls(t1, t2, L, r, legacy_wd_swap=legacy)
            out = blk(torch.from_numpy(coords).to(DEV))
            loss = (out * torch.from_numpy(G).to(DEV)).sum()
        # both blocks run the reference's fp16 (the materialised pyramid; the on-the-fly dots, round 4)
        assert blk.precision == "fp16" and out.dtype == torch.float32
        loss.backward()
        assert t1.grad.dtype == torch.float32 and t2.grad.dtype == torch.float32
        assert orc.rel_err(out.detach().cpu().numpy(), ref) <= BF16_TOL
        e1, e2 = orc.rel_err(t1.grad.cpu().numpy(), g["grad_f1"]), orc.rel_err(t2.grad.cpu().numpy(), g["grad_f2"])
        assert e1 <= BF16_TOL and e2 <= BF16_TOL, (cls.__name__, e1, e2)
    # outside autocast the same fp32 inputs build in exact f32; an explicit precision always wins
    assert dvccorr.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV), L, r).precision == "fp32"
    with torch.amp.autocast("cuda"):
        assert dvccorr.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV), L, r,
                                 precision="fp32").precision == "fp32"


def test_grad_reproducible_and_accumulates():
    """Bitwise reproducible (fixed summation order, no atomics); two lookups on one block (the GRU loop calls
    it 12x) accumulate like two independent calls."""
    import dvccorr
    H = W = D = 16
    C, L, r = 64, 3, 4
    f1 = torch.from_numpy(prng.normal(11, (1, C, H, W, D))).to(DEV)
    f2 = torch.from_numpy(prng.normal(12, (1, C, H, W, D))).to(DEV)
    cs = [torch.from_numpy(prng.flow_coords(13 + i, 1, H, W, D, 2.0)).to(DEV) for i in range(2)]
    Gs = [torch.from_numpy(prng.normal(20 + i, (1, L * (2 * r + 1) ** 3, H, W, D))).to(DEV) for i in range(2)]

    def run(which):
        t1, t2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
        blk = dvccorr.CorrBlock(t1, t2, L, r)
        loss = sum((blk(cs[i]) * Gs[i]).sum() for i in which)
        loss.backward()
        return t1.grad, t2.grad

    a1, a2 = run((0, 1))
    b1, b2 = run((0, 1))
    assert torch.equal(a1, b1) and torch.equal(a2, b2)
    p1, p2 = run((0,))
    q1, q2 = run((1,))
    assert orc.rel_err((p1 + q1).cpu().numpy(), a1.cpu().numpy()) < 1e-6
    assert orc.rel_err((p2 + q2).cpu().numpy(), a2.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("shape,C,L,r", [((8, 8, 4), 16, 2, 2), ((6, 16, 4), 8, 2, 4), ((7, 5, 17), 16, 3, 1),
                                         ((12, 9, 11), 32, 2, 6)])
def test_grad_legacy_w_ne_d(shape, C, L, r):
    """Legacy convention on levels with W != D (grid x/z normalised by one axis' size and unnormalised by the
    other's, corr.py:49-50): per-level window boxes of the stretched sample footprint (k_win_grad_generic),
    against autograd through the CPU restatement; ratios above and below 1, flows leaving the volume."""
    H, W, D = shape
    seed = 5000 + H * 100 + W * 10 + D + r
    f1 = prng.normal(seed, (1, C, H, W, D))
    f2 = prng.normal(seed + 1, (1, C, H, W, D))
    coords = prng.flow_coords(seed + 2, 1, H, W, D, r + 2.0)
    G = prng.normal(seed + 3, (1, L * (2 * r + 1) ** 3, H, W, D))
    ref1, ref2 = oracle_grads(f1, f2, coords, G, L, r, True)
    for kind in ("gemm", "fused"):
        d1, d2 = _gpu_grads(kind, f1, f2, coords, G, L, r, True)
        e1, e2 = orc.rel_err(d1, ref1), orc.rel_err(d2, ref2)
        assert e1 <= GRAD_TOL and e2 <= GRAD_TOL, (shape, r, kind, e1, e2)
    a1, a2 = _gpu_grads("gemm", f1, f2, coords, G, L, r, True)
    b1, b2 = _gpu_grads("gemm", f1, f2, coords, G, L, r, True)
    assert np.array_equal(a1, b1) and np.array_equal(a2, b2)


@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp16", FP16_TOL), ("fp32", GRAD_TOL)])
def test_grad_cfg3_slab(precision, tol):
    """Config #3 at full size (32^3, C = 128, L = 4, r = 4, +-2-voxel flows: the shape the backward is benchmarked
    at, so every size-dependent choice of the gradient kernels -- split counts sized by query count, the three-way
    level group of k_grad_q_mfma, the 8-aligned tile starts of k_tile_targets / k_qt_tiles -- runs as in the bench)
    with an output gradient that is nonzero on one ragged 512-row query slab only.  Against autograd through
    oracle/torch_cpu.py's build_rows / lookup_rows on that slab (corr.py:141-208 restated; rows are independent):
    d fmap1 on the slab rows, exact zeros elsewhere, d fmap2 in full."""
    import dvccorr
    from oracle import torch_cpu
    B, C, S, L, r = 1, 128, 32, 4, 4
    N, n3 = S ** 3, (2 * r + 1) ** 3
    q0, q1 = 12345, 12345 + 512
    f1 = prng.normal(7001, (B, C, S, S, S))
    f2 = prng.normal(7002, (B, C, S, S, S))
    coords = prng.flow_coords(7003, B, S, S, S, 2.0)
    Gs = prng.normal(7004, (B, L * n3, q1 - q0))
    # oracle: the slab's rows of every level, its lookup, autograd
    t1 = torch.from_numpy(f1).requires_grad_(True)
    t2 = torch.from_numpy(f2).requires_grad_(True)
    pyr = torch_cpu.build_rows(t1, t2, L, q0, q1)
    out = torch_cpu.lookup_rows(pyr, torch.from_numpy(coords), r, False, q0, q1)
    (out * torch.from_numpy(Gs)).sum().backward()
    ref1 = t1.grad.numpy().reshape(B, C, N)
    ref2 = t2.grad.numpy()
    # GPU: the whole block, G zero outside the slab
    g1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    g2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    blk = dvccorr.CorrBlock(g1, g2, L, r, precision=precision)
    G = torch.zeros((B, L * n3, N), device=DEV)
    G[:, :, q0:q1] = torch.from_numpy(Gs).to(DEV)
    (blk(torch.from_numpy(coords).to(DEV)) * G.view(B, L * n3, S, S, S)).sum().backward()
    d1 = g1.grad.reshape(B, C, N).cpu().numpy()
    d2 = g2.grad.cpu().numpy()
    assert np.isfinite(d1).all() and np.isfinite(d2).all()
    assert not d1[:, :, :q0].any() and not d1[:, :, q1:].any()
    e1 = orc.rel_err(d1[:, :, q0:q1], ref1[:, :, q0:q1])
    e2 = orc.rel_err(d2, ref2)
    assert e1 <= tol and e2 <= tol, (precision, e1, e2)


@pytest.mark.parametrize("precision,tol", [("fp32", GRAD_TOL), ("bf16", BF16_TOL), ("fp16", FP16_TOL)])
def test_grad_valu_fallback(precision, tol):
    """The VALU gradient kernels (k_grad_q / k_grad_t, 64-bit addressing): the path dvc_corr_backward takes for
    volumes past the matrix-core kernels' 31-bit buffer offsets (~154^3 level-0 fmaps and up, too large for a
    test), forced here with tuning "bwd_mfma" 0 on the C = 128, L = 4, r = 4 golden vectors (grad_cfg2)."""
    from dvccorr import _lib
    _lib.set_tuning("bwd_mfma", 0)
    try:
        _check_golden("grad_cfg2", "gemm", precision, tol)
    finally:
        _lib.set_tuning("bwd_mfma", 1)


@pytest.mark.parametrize("precision", ["bf16", "fp16", "fp32"])
def test_grad_gout64_instance(precision):
    """k_win_grad_pairs' 64-bit-addressed instance (the one volumes with more than 2^31 - 1 bytes per
    output-gradient row take, Nq > ~6.6 M at r = 4, too large for a test) forced with tuning "bwd_gout64" 1: the
    same gradients as the 32-bit-offset instance, bit for bit, and the golden vectors still pass."""
    from dvccorr import _lib, ops
    S, C, L, r = 12, 64, 3, 4
    seed = 515
    f1 = torch.from_numpy(prng.normal(seed, (1, C, S, S, S))).to(DEV)
    f2 = torch.from_numpy(prng.normal(seed + 1, (1, C, S, S, S))).to(DEV)
    coords = torch.from_numpy(prng.flow_coords(seed + 2, 1, S, S, S, 3.0)).to(DEV).reshape(1, 3, -1)
    G = torch.from_numpy(prng.normal(seed + 3, (1, L * (2 * r + 1) ** 3, S ** 3))).to(DEV)
    dt = ops.dtype_code(precision)
    q = ops.pack_queries(f1.reshape(1, C, -1), dt)
    t = ops.pack_targets(f2, L, dt)
    base = ops.corr_backward(q, t, coords, G, C, S, S, S, L, r, False, dt)
    _lib.set_tuning("bwd_gout64", 1)
    try:
        wide = ops.corr_backward(q, t, coords, G, C, S, S, S, L, r, False, dt)
        torch.cuda.synchronize()
        _check_golden("grad_cfg2", "gemm", precision, {"fp32": GRAD_TOL, "bf16": BF16_TOL, "fp16": FP16_TOL}[precision])
    finally:
        _lib.set_tuning("bwd_gout64", 0)
    for a, b in zip(base, wide):
        assert torch.equal(a, b)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_grad_stale_workspace(precision):
    """The window-gradient planes outside a level are never written (k_win_grad_pairs) and the 16-byte gradient
    reads of k_grad_q_mfma / k_grad_t_mfma straddle into neighbouring rows: no consumer may use such values.  The
    caching allocator is filled with NaN / -7 / 3e4 before each call, so the workspace holds stale values; the
    gradients (16^3, C = 128, L = 4, r = 4 with flows off the volume: coarse windows overhang their level) must be
    finite and bitwise equal across the three poisons."""
    from dvccorr import ops
    S, C, L, r = 16, 128, 4, 4
    seed = 4242
    f1 = torch.from_numpy(prng.normal(seed, (1, C, S, S, S))).to(DEV)
    f2 = torch.from_numpy(prng.normal(seed + 1, (1, C, S, S, S))).to(DEV)
    coords = torch.from_numpy(prng.flow_coords(seed + 2, 1, S, S, S, r + 3.0)).to(DEV).reshape(1, 3, -1)
    G = torch.from_numpy(prng.normal(seed + 3, (1, L * (2 * r + 1) ** 3, S ** 3))).to(DEV)
    dt = ops.dtype_code(precision)
    q = ops.pack_queries(f1.reshape(1, C, -1), dt)
    t = ops.pack_targets(f2, L, dt)
    nws = ops.lib().dvc_corr_backward_workspace_bytes(1, S ** 3, C, S, S, S, L, r)
    outs = []
    for val in (float("nan"), -7.0, 3.0e4):
        poison = torch.full((2 * nws // 4 + (1 << 20),), val, device=DEV)
        del poison
        d1, d2 = ops.corr_backward(q, t, coords, G, C, S, S, S, L, r, False, dt)
        torch.cuda.synchronize()
        assert bool(torch.isfinite(d1).all()) and bool(torch.isfinite(d2).all()), (precision, val)
        outs.append((d1.clone(), d2.clone()))
    for d1, d2 in outs[1:]:
        assert torch.equal(d1, outs[0][0]) and torch.equal(d2, outs[0][1]), precision


@pytest.mark.parametrize("shape,C,L,r,legacy,scale,B", [
    ((16, 16, 16), 64, 4, 4, False, 3.0, 1),    # config #2's pyramid: coarse cells of 8 / 64 / 512 queries
    ((8, 8, 8), 32, 4, 3, False, 2.0, 1),       # a one-voxel level: all its keys in the outside cell
    ((12, 10, 16), 32, 3, 4, False, 3.0, 2),    # ragged, two batch elements
    ((8, 12, 16), 32, 2, 2, True, 2.0, 1),      # legacy W != D: stretched windows (generic levels)
    ((24, 24, 24), 32, 2, 2, False, 60.0, 1),   # flows far off the volume: outside cells of > 4 K keys (unstaged)
])
def test_grad_counting_sort_matches_radix(shape, C, L, r, legacy, scale, B):
    """The target-gradient pass's counting sort (k_bw_keys' per-(wave, cell) slots, k_cell_scatter, k_cell_rank;
    round 5) against rocprim's stable radix sort + k_cell_starts (tuning "bwd_sort" 0): both gradients bit for bit,
    for every dtype, over the cell populations a sort meets -- near-empty level-0 cells, 512-query coarse cells,
    one-voxel levels, legacy stretched windows, a second batch element and outside cells holding most queries."""
    from dvccorr import _lib, ops
    H, W, D = shape
    seed = 8100 + H + 3 * L
    f1 = torch.from_numpy(prng.normal(seed, (B, C, H, W, D))).to(DEV)
    f2 = torch.from_numpy(prng.normal(seed + 1, (B, C, H, W, D))).to(DEV)
    coords = torch.from_numpy(prng.flow_coords(seed + 2, B, H, W, D, scale)).to(DEV).reshape(B, 3, -1)
    G = torch.from_numpy(prng.normal(seed + 3, (B, L * (2 * r + 1) ** 3, H * W * D))).to(DEV)
    for precision in ("bf16", "fp16", "fp32"):
        dt = ops.dtype_code(precision)
        q = ops.pack_queries(f1.reshape(B, C, -1), dt)
        t = ops.pack_targets(f2, L, dt)
        got = ops.corr_backward(q, t, coords, G, C, H, W, D, L, r, legacy, dt)
        _lib.set_tuning("bwd_sort", 0)
        try:
            ref = ops.corr_backward(q, t, coords, G, C, H, W, D, L, r, legacy, dt)
            torch.cuda.synchronize()
        finally:
            _lib.set_tuning("bwd_sort", 1)
        for a, b_ in zip(got, ref):
            assert torch.equal(a, b_), precision


@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp16", FP16_TOL)])
def test_grad_cfg4_slab(precision, tol):
    """Config #4 at full size (64^3 fmaps, C = 128, L = 4, r = 4, +-2-voxel flows; 262 K queries: the split counts,
    sorted groups, dense target batches and counting sort at 8x config #3's query count), on the on-the-fly block
    (the materialised 64^3 pyramid is 157 GB), with an output gradient nonzero on one ragged 512-row slab.  Against
    autograd through oracle/torch_cpu.py's build_rows / lookup_rows on that slab, as test_grad_cfg3_slab."""
    import dvccorr
    from oracle import torch_cpu
    B, C, S, L, r = 1, 128, 64, 4, 4
    N, n3 = S ** 3, (2 * r + 1) ** 3
    q0, q1 = 150001, 150001 + 512
    f1 = prng.normal(7101, (B, C, S, S, S))
    f2 = prng.normal(7102, (B, C, S, S, S))
    coords = prng.flow_coords(7103, B, S, S, S, 2.0)
    Gs = prng.normal(7104, (B, L * n3, q1 - q0))
    t1 = torch.from_numpy(f1).requires_grad_(True)
    t2 = torch.from_numpy(f2).requires_grad_(True)
    pyr = torch_cpu.build_rows(t1, t2, L, q0, q1)
    out = torch_cpu.lookup_rows(pyr, torch.from_numpy(coords), r, False, q0, q1)
    (out * torch.from_numpy(Gs)).sum().backward()
    ref1 = t1.grad.numpy().reshape(B, C, N)[:, :, q0:q1]
    ref2 = t2.grad.numpy()
    del pyr, out, t1, t2
    g1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    g2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    blk = dvccorr.CorrBlockFused(g1, g2, L, r, precision=precision)
    G = torch.zeros((B, L * n3, N), device=DEV)
    G[:, :, q0:q1] = torch.from_numpy(Gs).to(DEV)
    (blk(torch.from_numpy(coords).to(DEV)) * G.view(B, L * n3, S, S, S)).sum().backward()
    d1 = g1.grad.reshape(B, C, N)
    assert bool(torch.isfinite(d1).all()) and bool(torch.isfinite(g2.grad).all())
    assert not bool(d1[:, :, :q0].any()) and not bool(d1[:, :, q1:].any())
    e1 = orc.rel_err(d1[:, :, q0:q1].cpu().numpy(), ref1)
    e2 = orc.rel_err(g2.grad.cpu().numpy(), ref2)
    assert e1 <= tol and e2 <= tol, (precision, e1, e2)


@pytest.mark.parametrize("knobs", [{"bwd_dense": 0}, {"bwd_side": 0}, {"bwd_side_q": 0}, {"bwd_sort": 0},
                                   {"bwd_g16": 0, "bwd_dense": 0}])
@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp16", FP16_TOL), ("fp32", GRAD_TOL)])
def test_grad_round5_paths_off(knobs, precision, tol):
    """The round-5 backward paths switched off one at a time (tuning knobs, process-global since round 6, so the
    autograd engine's worker thread that runs this backward sees them too): the per-row target
    batches (k_qt_tiles + k_grad_t_mfma), the in-order stream, the dQ pass on the main stream, rocprim's radix sort,
    and the hi/lo window-gradient pairs -- each still passes the C = 128, L = 4, r = 4 golden vectors (grad_cfg2),
    so the fallbacks stay tested while the defaults move on."""
    from dvccorr import _lib
    defaults = {"bwd_dense": 1, "bwd_side": 1, "bwd_side_q": 1, "bwd_sort": 1, "bwd_g16": 1}
    for k, v in knobs.items():
        _lib.set_tuning(k, v)
    try:
        _check_golden("grad_cfg2", "gemm", precision, tol)
    finally:
        for k in knobs:
            _lib.set_tuning(k, defaults[k])


def test_tuning_reaches_the_autograd_thread():
    """the knobs were thread_local, so a backward run by PyTorch's autograd worker thread (loss.backward()
    on a CUDA graph) ignored a knob set by the caller.  With the knobs process-global, bwd_mfma 0 set here must select
    the VALU gradient kernels inside loss.backward(): the gradients equal ops.corr_backward's under the same knob on
    this thread bit for bit, and differ from the matrix-core defaults (another summation order)."""
    import dvccorr
    from dvccorr import _lib, ops
    S, C, L, r = 12, 64, 3, 3
    seed = 6060
    f1 = prng.normal(seed, (1, C, S, S, S))
    f2 = prng.normal(seed + 1, (1, C, S, S, S))
    coords = prng.flow_coords(seed + 2, 1, S, S, S, 2.5)
    G = prng.normal(seed + 3, (1, L * (2 * r + 1) ** 3, S, S, S))

    def autograd_grads():
        t1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
        t2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
        out = dvccorr.CorrBlock(t1, t2, L, r, precision="fp32")(torch.from_numpy(coords).to(DEV))
        (out * torch.from_numpy(G).to(DEV)).sum().backward()
        return t1.grad.reshape(1, C, -1), t2.grad

    dt = ops.dtype_code("fp32")
    q = ops.pack_queries(torch.from_numpy(f1).to(DEV).reshape(1, C, -1), dt)
    t = ops.pack_targets(torch.from_numpy(f2).to(DEV), L, dt)
    cg = torch.from_numpy(coords).to(DEV).reshape(1, 3, -1)
    gg = torch.from_numpy(G).to(DEV).reshape(1, -1, S ** 3)
    mfma = autograd_grads()
    _lib.set_tuning("bwd_mfma", 0)
    try:
        valu_ad = autograd_grads()
        valu_direct = ops.corr_backward(q, t, cg, gg, C, S, S, S, L, r, False, dt)
        torch.cuda.synchronize()
    finally:
        _lib.set_tuning("bwd_mfma", 1)
    for a, b in zip(valu_ad, valu_direct):
        assert torch.equal(a, b)
    assert not torch.equal(mfma[1], valu_ad[1]), "the knob did not reach the autograd thread"


@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp32", GRAD_TOL)])
def test_grad_zero_level_outside_cell(precision, tol):
    """Verdict r5: a (64, 64, 8) fmap at C = 128, L = 4, r = 4 (a 256 x 256 x 32 volume at 1/4) has a size-1 level 3
    ((8, 8, 1), a "zero" level): all 32 K of its keys fall in that level's outside cell, which the counting sort ranked
    by re-reading the whole cell from memory per key (~1e9 loads).  Outside cells now keep their arrival order (no
    gradient reads them).  Checked: the gradients against autograd through oracle/torch_cpu.py on a ragged 512-row
    slab (as test_grad_cfg3_slab), and the backward's time per query within 2x config #3's (32^3, the same 32 K
    queries, no zero level)."""
    import dvccorr
    from dvccorr import ops
    from oracle import torch_cpu
    B, C, L, r = 1, 128, 4, 4
    H, W, D = 64, 64, 8
    N, n3 = H * W * D, (2 * r + 1) ** 3
    q0, q1 = 20001, 20001 + 512
    f1 = prng.normal(7201, (B, C, H, W, D))
    f2 = prng.normal(7202, (B, C, H, W, D))
    coords = prng.flow_coords(7203, B, H, W, D, 2.0)
    Gs = prng.normal(7204, (B, L * n3, q1 - q0))
    t1 = torch.from_numpy(f1).requires_grad_(True)
    t2 = torch.from_numpy(f2).requires_grad_(True)
    pyr = torch_cpu.build_rows(t1, t2, L, q0, q1)
    out = torch_cpu.lookup_rows(pyr, torch.from_numpy(coords), r, False, q0, q1)
    (out * torch.from_numpy(Gs)).sum().backward()
    ref1 = t1.grad.numpy().reshape(B, C, N)[:, :, q0:q1]
    ref2 = t2.grad.numpy()
    g1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    g2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    blk = dvccorr.CorrBlock(g1, g2, L, r, precision=precision)
    G = torch.zeros((B, L * n3, N), device=DEV)
    G[:, :, q0:q1] = torch.from_numpy(Gs).to(DEV)
    (blk(torch.from_numpy(coords).to(DEV)) * G.view(B, L * n3, H, W, D)).sum().backward()
    d1 = g1.grad.reshape(B, C, N)
    assert bool(torch.isfinite(d1).all()) and bool(torch.isfinite(g2.grad).all())
    assert not bool(d1[:, :, :q0].any()) and not bool(d1[:, :, q1:].any())
    e1 = orc.rel_err(d1[:, :, q0:q1].cpu().numpy(), ref1)
    e2 = orc.rel_err(g2.grad.cpu().numpy(), ref2)
    assert e1 <= tol and e2 <= tol, (precision, e1, e2)

    # time per query against config #3's shape (same query count)
    def bwd_ms(shape, seed):
        h, w, d = shape
        dt = ops.dtype_code(precision)
        a = torch.from_numpy(prng.normal(seed, (1, C, h, w, d))).to(DEV)
        b = torch.from_numpy(prng.normal(seed + 1, (1, C, h, w, d))).to(DEV)
        c = torch.from_numpy(prng.flow_coords(seed + 2, 1, h, w, d, 2.0)).to(DEV).reshape(1, 3, -1)
        g = torch.randn((1, L * n3, h * w * d), device=DEV)
        q = ops.pack_queries(a.reshape(1, C, -1), dt)
        t = ops.pack_targets(b, L, dt)
        ops.corr_backward(q, t, c, g, C, h, w, d, L, r, False, dt)
        torch.cuda.synchronize()
        e0, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.corr_backward(q, t, c, g, C, h, w, d, L, r, False, dt)
        e1_.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1_) / 3

    t_zero = bwd_ms((H, W, D), 7301)
    t_cfg3 = bwd_ms((32, 32, 32), 7311)
    assert t_zero <= 2.0 * t_cfg3, (precision, t_zero, t_cfg3)


def test_graph_captured_backward():
    """dvc_corr_backward captured in a HIP graph (torch.cuda.CUDAGraph over the C ABI; while the stream is being
    captured the backward keeps every launch on it instead of forking its side stream) and replayed twice, the second
    time on a new output gradient, gives the eager (side-stream) gradients bit for bit.  (Round 5: with the zero guard
    and the cell counts cleared by hipMemsetAsync, replays after the first returned garbage d fmap2 -- the clears are
    kernels now, common.h zero_async.)"""
    from dvccorr import ops
    S, C, L, r = 16, 64, 4, 4
    f1 = torch.from_numpy(prng.normal(950, (1, C, S, S, S))).to(DEV)
    f2 = torch.from_numpy(prng.normal(951, (1, C, S, S, S))).to(DEV)
    coords = torch.from_numpy(prng.flow_coords(952, 1, S, S, S, 2.0)).to(DEV).reshape(1, 3, -1)
    G = torch.from_numpy(prng.normal(953, (1, L * (2 * r + 1) ** 3, S ** 3))).to(DEV)
    dt = ops.dtype_code("bf16")
    q = ops.pack_queries(f1.reshape(1, C, -1), dt)
    t = ops.pack_targets(f2, L, dt)
    run = lambda g: ops.corr_backward(q, t, coords, g, C, S, S, S, L, r, False, dt)   # noqa: E731
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run(G)   # warm-up outside capture
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g1, g2 = run(G)
    graph.replay()
    G.copy_(torch.from_numpy(prng.normal(954, tuple(G.shape))).to(DEV))
    graph.replay()   # (a second replay: the clears of the zero guard and the cell counts must run again)
    torch.cuda.synchronize()
    e1, e2 = run(G)
    torch.cuda.synchronize()
    assert torch.equal(g1, e1) and torch.equal(g2, e2)


@pytest.mark.gpu
def test_graph_captured_backward_poisoned_workspace():
    """A caller-owned workspace filled with NaN before the capture and again between replays: every replay clears
    what it needs (the zero guard, the cell counts) itself, so the replayed gradients equal the eager ones bit for
    bit and the guard reads zero after each replay (tools/graph_bwd_diag.py's check, round 5)."""
    from dvccorr import ops
    from dvccorr.ops import _ptr, _stream, lib
    S, C, L, r = 16, 64, 4, 4
    B, Nq = 1, S ** 3
    f1 = torch.from_numpy(prng.normal(960, (1, C, S, S, S))).to(DEV)
    f2 = torch.from_numpy(prng.normal(961, (1, C, S, S, S))).to(DEV)
    coords = torch.from_numpy(prng.flow_coords(962, 1, S, S, S, 2.0)).to(DEV).reshape(1, 3, -1).contiguous()
    G = torch.from_numpy(prng.normal(963, (1, L * (2 * r + 1) ** 3, Nq))).to(DEV).contiguous()
    dt = ops.dtype_code("bf16")
    q = ops.pack_queries(f1.reshape(1, C, -1), dt)
    t = ops.pack_targets(f2, L, dt)
    nws = lib().dvc_corr_backward_workspace_bytes_dtype(B, Nq, C, S, S, S, L, r, dt)
    ws = torch.full((nws // 4 + 64,), float("nan"), device=DEV)
    d1 = torch.empty((B, C, Nq), device=DEV)
    d2 = torch.empty((B, C, S, S, S), device=DEV)
    e1, e2 = ops.corr_backward(q, t, coords, G, C, S, S, S, L, r, False, dt)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=torch.cuda.Stream()):
        ops.check(lib().dvc_corr_backward(_ptr(q), _ptr(t), _ptr(coords), _ptr(G), _ptr(d1), _ptr(d2), _ptr(ws), B,
                                          Nq, C, S, S, S, L, r, 0, dt, _stream(q)), "corr_backward")
    for _ in range(2):
        ws.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert bool((ws[:64] == 0).all())
        assert torch.equal(d1, e1) and torch.equal(d2, e2)
