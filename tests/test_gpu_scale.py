"""GPU parity at BASELINE configs #4 and #5 (the sizes the bench and the north star name),
plus the boundary features added in round 2.

  #4  256^3 input, 1/4 encoder: 64^3 x 128 fmaps, L=4, r=4, bf16.  One rank's 8-plane
      H-slab of an 8-way query-voxel split (dvccorr.sharded.HipRows: the per-rank compute of
      ShardedCorrBlock) equals the same rows of the whole-grid CorrBlock bit for bit, and
      sampled rows match the f64 oracle (<= 1e-2, bf16 build).   corr.py:116-208
  #5  256^3 input, 1/2 encoder: 128^3 x 128 fmaps, L=2, r=4, on-the-fly (no volume):
      sampled rows of CorrBlockFused against the f64 oracle (<= 1e-2).   corr_otf.py:96-237

Inputs at these sizes come from torch's GPU generator (seeded); the oracle reads the same
values copied back to the host, so no fixture is needed.  Tolerance: max|out-ref|/max|ref|.
"""
from __future__ import annotations

import gc

import numpy as np
import pytest
import torch

import prng
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
BF16_TOL = 1e-2
FP32_TOL = 1e-5


@pytest.fixture(autouse=True)
def _free():
    yield
    gc.collect()
    torch.cuda.empty_cache()


def _inputs(seed, C, S, max_flow=2.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    f1 = torch.randn(1, C, S, S, S, device=DEV, generator=g)
    f2 = torch.randn(1, C, S, S, S, device=DEV, generator=g)
    base = torch.stack(torch.meshgrid(*[torch.arange(S, device=DEV, dtype=torch.float32)] * 3, indexing="ij"))
    c = base[None] + (torch.rand(1, 3, S, S, S, device=DEV, generator=g) * 2 - 1) * max_flow
    return f1, f2, c.contiguous()


def _oracle_rows(f1, f2, c, L, r, rows, legacy=False):
    return orc.corr_lookup(f1.cpu().numpy(), f2.cpu().numpy(), c.cpu().numpy(), L, r, legacy, rows=rows)


def _rows(out_flat, rows):
    """out_flat (1, K, N) -> [len(rows), K]."""
    idx = torch.as_tensor(rows, device=out_flat.device)
    return out_flat[0][:, idx].t().float().cpu().numpy()


@pytest.mark.parametrize("rank", [0, 5])
def test_cfg4_rank_slab(rank):
    """Config #4: rank `rank` of an 8-way H-slab split (8 of 64 planes, 32768 query rows) is the same
    rows of the whole-grid materialised block, bit for bit, and matches the oracle on sampled rows."""
    import dvccorr
    from dvccorr.sharded import HipRows, slab_bounds
    S, C, L, r, world = 64, 128, 4, 4, 8
    f1, f2, c = _inputs(404, C, S)
    h0, h1 = slab_bounds(S, world, rank)
    with torch.no_grad():
        blk = dvccorr.CorrBlock(f1, f2, L, r, precision="bf16")          # 157 GB pyramid
        full = blk(c).reshape(1, L * (2 * r + 1) ** 3, S, S, S)[:, :, h0:h1].contiguous()
        del blk
        gc.collect()
        torch.cuda.empty_cache()
        rows = HipRows(f1[:, :, h0:h1].reshape(1, C, -1), f2, L, r, False, "bf16", "materialised")
        part = rows.lookup(c[:, :, h0:h1].reshape(1, 3, -1).contiguous())
        torch.cuda.synchronize()
    assert torch.equal(part.view_as(full), full)
    assert torch.isfinite(part).all()
    n = (h1 - h0) * S * S
    local = np.sort(np.random.default_rng(4040 + rank).choice(n, 48, replace=False)).astype(np.int64)
    ref = _oracle_rows(f1, f2, c, L, r, local + h0 * S * S)
    assert orc.rel_err(_rows(part, local), ref) <= BF16_TOL


FP16_TOL = 5e-3     # the reference's AMP tolerance (test_corr_equivalence.py:156-186)


@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp16", FP16_TOL), ("fp32", FP32_TOL)])
def test_cfg5_fused_rows(precision, tol):
    """Config #5: 128^3 x 128 fmaps, L=2, r=4, on-the-fly block (the 9.9 TB volume is never built):
    256 sampled query rows (plus corners, edges and one chunk's lanes 48-63) against the f64 oracle at the
    operand dtype's tolerance -- bf16 (the bench's dtype), fp16 (the Trainer's AMP operands) and fp32 (the
    reference's evaluation dtype; round 6: on the matrix cores, k_fused_box_f32)."""
    import dvccorr
    S, C, L, r = 128, 128, 2, 4
    f1, f2, c = _inputs(505, C, S)
    with torch.no_grad():
        blk = dvccorr.CorrBlockFused(f1, f2, L, r, precision=precision)
        out = blk(c).reshape(1, L * (2 * r + 1) ** 3, -1)
        torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    N = S ** 3
    rows = np.sort(np.random.default_rng(505).choice(N, 256, replace=False))
    rows = np.unique(np.concatenate([rows, [0, N - 1, S - 1, S * S - 1, S * S * 64 + S * 3 + 127,
                                            4096 + 48, 4096 + 63]])).astype(np.int64)
    ref = _oracle_rows(f1, f2, c, L, r, rows)
    assert orc.rel_err(_rows(out, rows), ref) <= tol
    if precision != "bf16":
        return
    # the same kernels, a slab of queries (the sharded #5 layout) is the slab of the whole result
    from dvccorr.sharded import HipRows
    with torch.no_grad():
        part = HipRows(f1[:, :, 48:64].reshape(1, C, -1), f2, L, r, False, "bf16", "fused").lookup(
            c[:, :, 48:64].reshape(1, 3, -1).contiguous())
    assert torch.equal(part, out[:, :, 48 * S * S:64 * S * S])


def test_cfg5_fused_convc1_rows():
    """Config #5 with MotionEncoder.convc1 fused (dvc_corr_lookup_fused_proj: k_otf_keys + radix sort +
    k_fused_proj + k_rows_to_channels) at full size, 128^3 x 128 fmaps, L=2, r=4, bf16: sampled query
    rows of relu(convc1(lookup)) against the f64 oracle at the bf16 tolerance (update.py:222, 246;
    corr_otf.py:198-237), and two calls bitwise equal (the kernel whose packed-FP32 broadcasts once
    corrupted lanes 48-63 intermittently)."""
    import dvccorr
    S, C, L, r = 128, 128, 2, 4
    f1, f2, c = _inputs(515, C, S)
    K = L * (2 * r + 1) ** 3
    g = torch.Generator(device="cpu").manual_seed(516)
    w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(DEV)
    b = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(DEV)
    with torch.no_grad():
        blk = dvccorr.CorrBlockFused(f1, f2, L, r, precision="bf16")
        out = blk.lookup_convc1(c, w, b).reshape(1, 96, -1)
        out2 = blk.lookup_convc1(c, w, b).reshape(1, 96, -1)
        torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert torch.equal(out, out2)
    N = S ** 3
    rows = np.sort(np.random.default_rng(515).choice(N, 32, replace=False))
    # plus the volume's corners/edges and rows inside one 64-query chunk's lanes 48-63
    rows = np.unique(np.concatenate([rows, [0, N - 1, S - 1, S * S * 64 + S * 3 + 127, 4096 + 48, 4096 + 63]]))
    rows = rows.astype(np.int64)
    look = _oracle_rows(f1, f2, c, L, r, rows)                                   # [rows, K] f64
    ref = np.maximum(look @ w.cpu().double().numpy().T + b.cpu().double().numpy()[None], 0.0)
    assert orc.rel_err(_rows(out, rows), ref) <= BF16_TOL


@pytest.mark.parametrize("precision,tol", [("bf16", BF16_TOL), ("fp32", FP32_TOL)])
def test_wide_features_c256(precision, tol):
    """C = 256 (C_pad 256): the bf16 build instances whose spilled prefetch registers faulted in round 1
    (now compiler-visible loads), the K-chunked exact-f32 build, and the on-the-fly block."""
    import dvccorr
    B, C, H, W, D, L, r = 1, 256, 12, 10, 14, 3, 3
    f1 = prng.normal(2561, (B, C, H, W, D))
    f2 = prng.normal(2562, (B, C, H, W, D))
    coords = prng.flow_coords(2563, B, H, W, D, 3.0)
    ref = orc.corr_lookup(f1, f2, coords, L, r, False)
    t1, t2, tc = (torch.from_numpy(a).to(DEV) for a in (f1, f2, coords))
    with torch.no_grad():
        out = dvccorr.CorrBlock(t1, t2, L, r, precision=precision)(tc)
        fz = dvccorr.CorrBlockFused(t1, t2, L, r, precision=precision)(tc)
        torch.cuda.synchronize()
    assert orc.rel_err(out.cpu().numpy(), ref) <= tol
    assert orc.rel_err(fz.cpu().numpy(), ref) <= tol


def test_capacity_check_and_auto_impl():
    """A pyramid larger than the free HBM raises OutOfMemoryError before anything is allocated
    (the reference Trainer catches it, trainer.py:287-304); mi355x_auto picks the fused block."""
    import dvccorr
    f = torch.randn(1, 32, 96, 96, 96, device=DEV)       # 96^6 x 2 B = 1.6 TB pyramid at L=1
    before = torch.cuda.memory_allocated(DEV)
    with pytest.raises(torch.cuda.OutOfMemoryError, match="CorrBlockFused"):
        dvccorr.CorrBlock(f, f, 1, 4, precision="bf16")
    assert torch.cuda.memory_allocated(DEV) == before
    blk = dvccorr.make_corr_block("mi355x_auto", f, f, 1, 4, precision="bf16")
    assert isinstance(blk, dvccorr.CorrBlockFused)
    # CorrBlock-only keywords are dropped on the fallback (they raised TypeError exactly there)
    blk = dvccorr.make_corr_block("mi355x_auto", f, f, 1, 4, precision="bf16", build="gemm", bricked=True)
    assert isinstance(blk, dvccorr.CorrBlockFused)
    small = torch.randn(1, 32, 8, 8, 8, device=DEV)
    assert type(dvccorr.make_corr_block("mi355x_auto", small, small, 2, 2)) is dvccorr.CorrBlock


def test_checkpointed_lookup_matches():
    """torch.utils.checkpoint(block, coords, use_reentrant=False) -- the reference's checkpoint_corr path
    (raft_dvc.py:446-448) -- gives the same forward values and the same fmap gradients bit for bit."""
    import dvccorr
    from torch.utils.checkpoint import checkpoint
    B, C, H, W, D, L, r = 1, 64, 10, 12, 8, 3, 3
    g = torch.Generator(device="cpu").manual_seed(3)
    a = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    b = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    cs = [torch.from_numpy(prng.flow_coords(30 + i, B, H, W, D, 2.0)).to(DEV) for i in range(3)]
    wts = [torch.randn(B, L * (2 * r + 1) ** 3, H, W, D, generator=g).to(DEV) for _ in range(3)]
    grads, outs = [], []
    for ck in (False, True):
        for impl in ("mi355x", "mi355x_fused"):
            f1 = a.clone().requires_grad_(True)
            f2 = b.clone().requires_grad_(True)
            blk = dvccorr.make_corr_block(impl, f1, f2, L, r)
            loss = 0
            for c, w in zip(cs, wts):
                o = checkpoint(blk, c, use_reentrant=False) if ck else blk(c)
                loss = loss + (o * w).sum()
            loss.backward()
            outs.append(loss.detach())
            grads.append((f1.grad.clone(), f2.grad.clone()))
    for i in (0, 1):
        assert torch.equal(outs[i], outs[i + 2])
        assert torch.equal(grads[i][0], grads[i + 2][0]) and torch.equal(grads[i][1], grads[i + 2][1])


def test_custom_ops_opcheck():
    """The torch.library registrations (dvccorr::build / lookup / lookup_fused / corr_backward / lookup_ad):
    schema, fake (meta) shapes and the autograd registration checked by torch.library.opcheck."""
    from dvccorr import ops
    B, C, H, W, D, L, r = 1, 32, 8, 9, 10, 2, 2
    g = torch.Generator(device="cpu").manual_seed(9)
    f1 = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    c = torch.from_numpy(prng.flow_coords(91, B, H, W, D, 2.0)).to(DEV).reshape(B, 3, -1)
    dt = ops.dtype_code("fp32")
    q = ops.pack_queries(f1.reshape(B, C, -1), dt)
    t = ops.pack_targets(f2, L, dt)
    corr = torch.ops.dvccorr.build(q, t, C, H, W, D, L, dt)
    tests = ("test_schema", "test_faketensor", "test_aot_dispatch_dynamic")
    torch.library.opcheck(torch.ops.dvccorr.build, (q, t, C, H, W, D, L, dt), test_utils=tests)
    torch.library.opcheck(torch.ops.dvccorr.lookup, (corr, c, H, W, D, L, r, False, dt), test_utils=tests)
    torch.library.opcheck(torch.ops.dvccorr.lookup_fused, (q, t, c, C, H, W, D, L, r, False, dt), test_utils=tests)
    f1g, f2g = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    torch.library.opcheck(torch.ops.dvccorr.lookup_ad, (f1g, f2g, corr, q, t, c, C, H, W, D, L, r, False, dt),
                          test_utils=tests + ("test_autograd_registration",))


def test_flow_step_gradients():
    """flow_step / upflow_3d are differentiable like the reference's tail (raft_dvc.py:482-486): the loss on
    flow_up reaches delta_flow.  Gradients against autograd through the reference formula (GPU torch ops)."""
    import dvccorr
    import torch.nn.functional as F
    B, h, w, d = 1, 6, 7, 5
    T = (24, 28, 20)
    g = torch.Generator(device="cpu").manual_seed(4)
    c1 = torch.from_numpy(prng.flow_coords(44, B, h, w, d, 1.0)).to(DEV)
    delta = (torch.randn(B, 3, h, w, d, generator=g) * 0.3).to(DEV)
    gu = torch.randn(B, 3, *T, generator=g).to(DEV)
    gc1 = torch.randn(B, 3, h, w, d, generator=g).to(DEV)

    def ref_tail(c, dl):
        c = c + dl
        up = F.interpolate(c - dvccorr.coords_grid_3d(B, h, w, d, DEV), size=T, mode="trilinear", align_corners=True)
        up = up * torch.tensor([T[0] / h, T[1] / w, T[2] / d], device=DEV).view(1, 3, 1, 1, 1)
        return c, up

    outs = []
    for fn in (dvccorr.flow_step, ref_tail):
        c = c1.clone().requires_grad_(True)
        dl = delta.clone().requires_grad_(True)
        nc, up = fn(c, dl) if fn is ref_tail else fn(c, dl, T)
        ((up * gu).sum() + (nc * gc1).sum()).backward()
        outs.append((up.detach(), c.grad, dl.grad))
    assert orc.rel_err(outs[0][0].cpu().numpy(), outs[1][0].cpu().numpy()) <= FP32_TOL
    for k in (1, 2):
        assert orc.rel_err(outs[0][k].cpu().numpy(), outs[1][k].cpu().numpy()) <= FP32_TOL
    # upflow_3d alone, uncertainty-style (C = 3)
    f = delta.clone().requires_grad_(True)
    dvccorr.upflow_3d(f, T).mul(gu).sum().backward()
    f_ref = delta.clone().requires_grad_(True)
    up = F.interpolate(f_ref, size=T, mode="trilinear", align_corners=True)
    (up * torch.tensor([T[0] / h, T[1] / w, T[2] / d], device=DEV).view(1, 3, 1, 1, 1) * gu).sum().backward()
    assert orc.rel_err(f.grad.cpu().numpy(), f_ref.grad.cpu().numpy()) <= FP32_TOL
    with pytest.raises(NotImplementedError):
        dvccorr.bilinear_sampler_3d(torch.ones(1, 1, 4, 4, 4, device=DEV, requires_grad=True),
                                    torch.zeros(1, 2, 2, 2, 3, device=DEV))


def test_proj_pack_cache_tracks_the_weight_object():
    """A new convc1 weight allocated where a freed one lived (same address, same version counter) is
    re-packed: the cache belongs to the tensor object, not its address."""
    import dvccorr
    B, C, H, W, D, L, r = 1, 32, 8, 8, 8, 2, 2
    K = L * (2 * r + 1) ** 3
    g = torch.Generator(device="cpu").manual_seed(12)
    f1 = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    f2 = torch.randn(B, C, H, W, D, generator=g).to(DEV)
    c = torch.from_numpy(prng.flow_coords(121, B, H, W, D, 2.0)).to(DEV)
    blk = dvccorr.CorrBlock(f1, f2, L, r, precision="bf16")
    bias = torch.zeros(96, device=DEV)
    with torch.no_grad():
        w1 = torch.full((96, K), 0.01, device=DEV)
        o1 = blk.lookup_convc1(c, w1, bias)
        del w1
        w2 = torch.full((96, K), -0.02, device=DEV)
        o2 = blk.lookup_convc1(c, w2, bias)
        ref2 = torch.relu(torch.nn.functional.conv3d(blk(c), w2.view(96, K, 1, 1, 1), bias))
    assert not torch.equal(o1, o2)            # whether or not w2 reused w1's block (addr)
    assert orc.rel_err(o2.cpu().numpy(), ref2.cpu().numpy()) <= BF16_TOL


def test_fp32_block_convc1_is_exact():
    """convc1 on an fp32 block keeps fp32 arithmetic (<= 1e-5 against the f64 oracle of the reference's
    relu(convc1(corr)), update.py:246); bf16 blocks use the fused bf16-MFMA kernel (<= 1e-2)."""
    import dvccorr
    B, C, H, W, D, L, r = 1, 64, 8, 9, 10, 2, 4
    f1 = prng.normal(71, (B, C, H, W, D))
    f2 = prng.normal(72, (B, C, H, W, D))
    coords = prng.flow_coords(73, B, H, W, D, 2.0)
    K = L * (2 * r + 1) ** 3
    w = prng.uniform(74, (96, K), -K ** -0.5, K ** -0.5)
    bias = prng.uniform(75, (96,), -K ** -0.5, K ** -0.5)
    ref = orc.motion_convc1(orc.corr_lookup(f1, f2, coords, L, r, False), w, bias)
    t1, t2, tc, tw, tb = (torch.from_numpy(a).to(DEV) for a in (f1, f2, coords, w, bias))
    with torch.no_grad():
        e32 = orc.rel_err(dvccorr.CorrBlock(t1, t2, L, r).lookup_convc1(tc, tw, tb).cpu().numpy(), ref)
        e16 = orc.rel_err(dvccorr.CorrBlock(t1, t2, L, r, precision="bf16").lookup_convc1(tc, tw, tb).cpu().numpy(),
                          ref)
    assert e32 <= FP32_TOL, e32
    assert e16 <= BF16_TOL, e16


@pytest.mark.parametrize("shape,C,L", [((9, 7, 8), 16, 3), ((16, 16, 16), 128, 4), ((33, 20, 17), 40, 4),
                                       ((8, 8, 2), 64, 2), ((5, 6, 7), 32, 1), ((32, 32, 32), 128, 4),
                                       ((24, 18, 40), 256, 4), ((64, 64, 64), 128, 4), ((96, 64, 37), 160, 3)])
def test_single_pass_pack_matches_per_level(shape, C, L):
    """k_pack_pyramid (fmap2 -> every packed target level in one pass, pooled in LDS) writes exactly the
    bytes of the per-level pool + pack launches (same (dy, dx, dz) summation order), both dtypes.  The last
    two shapes have >= 2048 (cell, 32-channel group) pairs: the 32-channel instance."""
    from dvccorr import _lib, ops
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(H + W + D + C + L)
    f2 = torch.randn(2, C, H, W, D, generator=g).to(DEV)
    lay = ops.layout(H, W, D, L, C)
    for prec in ("bf16", "fp32"):
        dt = ops.dtype_code(prec)
        try:
            _lib.set_tuning("pack_variant", 0)
            old = ops.pack_targets(f2, L, dt)
        finally:
            _lib.set_tuning("pack_variant", 1)
        for cg in (0, 8, 16, 32):   # channels per workgroup: by size (0), or forced (tuning "pack_cg")
            # every row (voxels, z padding, the tail up to row_stride) must be written: start from NaN
            new = torch.full((2, lay.row_stride, lay.c_pad), float("nan"), dtype=ops._TORCH_DT[dt], device=DEV)
            try:
                _lib.set_tuning("pack_cg", cg)
                ops.pack_targets(f2, L, dt, out=new)
            finally:
                _lib.set_tuning("pack_cg", 0)
            torch.cuda.synchronize()
            assert torch.equal(new, old), (shape, C, L, prec, cg)


@pytest.mark.parametrize("shape,C,L,world", [((32, 32, 32), 128, 4, 8), ((32, 32, 32), 128, 4, 1),
                                             ((33, 20, 17), 40, 4, 5), ((16, 16, 16), 64, 3, 3),
                                             ((9, 7, 8), 16, 2, 9), ((64, 24, 40), 256, 4, 7)])
def test_pack_targets_gathered_matches_assembled(shape, C, L, world):
    """dvc_pack_targets_gathered (the targets packed straight from an H-slab all-gather's receive buffer, the
    multi-GPU forward) writes exactly the bytes of dvc_pack_targets on the assembled fmap2: balanced splits with
    and without a remainder (padded slabs), one plane per rank, B = 2, every dtype, bricked levels."""
    from dvccorr import ops
    from dvccorr.sharded import assemble_slabs, slab_bounds
    from dvccorr.corr_block import brick_flag
    H, W, D = shape
    g = torch.Generator(device="cpu").manual_seed(H * W + D + C + L + world)
    f2 = torch.randn(2, C, H, W, D, generator=g).to(DEV)
    maxh = -(-H // world)
    buf = torch.full((world, 2, C, maxh, W, D), float("nan"), device=DEV)   # pad planes must never be read
    for r in range(world):
        h0, h1 = slab_bounds(H, world, r)
        buf[r, :, :, :h1 - h0] = f2[:, :, h0:h1]
    assert torch.equal(assemble_slabs(torch.nan_to_num(buf), H), f2)
    lay = ops.layout(H, W, D, L, C)
    for prec in ("bf16", "fp16", "fp32"):
        for brick in (0, brick_flag(lay, 4, False, True)):
            dt = ops.dtype_code(prec) | brick
            got = ops.pack_targets_gathered(buf, H, L, dt)
            ref = ops.pack_targets(f2, L, dt)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), (shape, C, L, world, prec, brick)


@pytest.mark.parametrize("impl", ["materialised", "fused"])
def test_hiprows_gathered_lookup_matches(impl):
    """One rank's HipRows built from the all-gather buffer (gathered=) looks up the same values, bit for bit, as
    HipRows on the assembled fmap2 (config #3's 8-way slab, bf16), materialised and on the fly."""
    from dvccorr.sharded import HipRows, slab_bounds
    S, C, L, r, world, rank = 32, 128, 4, 4, 8, 3
    f1, f2, c = _inputs(77, C, S)
    h0, h1 = slab_bounds(S, world, rank)
    buf = torch.zeros((world, 1, C, -(-S // world), S, S), device=DEV)
    for k in range(world):
        a, b = slab_bounds(S, world, k)
        buf[k, :, :, :b - a] = f2[:, :, a:b]
    q = f1[:, :, h0:h1].reshape(1, C, -1).contiguous()
    cs = c[:, :, h0:h1].reshape(1, 3, -1).contiguous()
    with torch.no_grad():
        ref = HipRows(q, f2, L, r, False, "bf16", impl, q_offset=h0 * S * S).lookup(cs)
        got = HipRows(q, None, L, r, False, "bf16", impl, q_offset=h0 * S * S, gathered=(buf, S)).lookup(cs)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
