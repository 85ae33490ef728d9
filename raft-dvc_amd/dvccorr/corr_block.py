"""Drop-in correlation blocks for RAFT-DVC on MI355X.

Same constructor and call contract as the reference (zachtong/RAFT-DVC):

    CorrBlock(fmap1, fmap2, num_levels=4, radius=4, legacy_wd_swap=False)   src/core/corr.py:116-139
    CorrBlock.__call__(coords) -> (B, num_levels*(2r+1)**3, H, W, D) fp32    src/core/corr.py:169-208
    CorrBlockOnTheFly(fmap1, fmap2, num_levels, radius, chunk_size,
                      use_checkpoint)                                         src/core/corr_otf.py:51-94
    bilinear_sampler_3d(vol, coords, legacy_wd_swap=False)                    src/core/corr.py:17-68
    coords_grid_3d(batch, ht, wd, dp, device)                                 src/core/corr.py:71-99
    upflow_3d(flow, target_shape=None, scale_factor=8)                        src/core/corr.py:211-253
    flow_step(coords1, delta_flow, target_shape) -> (coords1', flow_up)       src/core/raft_dvc.py:482-485

so RAFTDVC.forward (raft_dvc.py:369-450), the trainer and the evaluation
scripts can use them unchanged.  The work is done by libdvccorr.so (gfx950
HIP kernels): an MFMA GEMM builds every pyramid level against the pooled
target features (equal to pooling the correlation, corr_otf.py:80-86), the
lookup is a lane-per-query gather kernel, and the on-the-fly block never
materialises the O(N^2) volume.

Precision: fp32 feature maps build in exact f32 MFMA and store fp32
(tolerance 1e-5 relative to the reference); `precision="bf16"` builds on
bf16 MFMA and stores bf16 (tolerance 1e-2), halving the HBM traffic;
`precision="fp16"` builds on fp16 MFMA and stores fp16 -- the reference's
pyramid under its Trainer's autocast, and the default inside an enabled CUDA
autocast region; otherwise the default follows the input dtype (fp16 -> fp16,
bf16 -> bf16), overridable with the DVCCORR_PRECISION environment variable.

Backward: when a feature map requires grad, every call is the differentiable
operator dvccorr::lookup_ad (library.py) whose registered autograd formula runs
dvc_corr_backward (sparse per-query window gradients, no dense d(corr), no
atomics) and returns d fmap1 / d fmap2; coordinates get no gradient, as
RAFTDVC.forward detaches them (raft_dvc.py:441).  Twelve calls on one block
accumulate in autograd like the reference's twelve grid_sample calls, and
torch.utils.checkpoint(block, coords, use_reentrant=False) (checkpoint_corr,
raft_dvc.py:446-448) recomputes the lookup in the backward pass.

Capacity: the materialised pyramid is B * N * row_stride values; CorrBlock
checks it against the device's free HBM before allocating and raises
torch.cuda.OutOfMemoryError naming the on-the-fly block instead (the
reference's Trainer catches that error, trainer.py:287-304);
make_corr_block("mi355x_auto", ...) picks the fused block when the volume
does not fit.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from . import library, ops
from ._lib import layout

__all__ = ["CorrBlock", "CorrBlockFused", "CorrBlockOnTheFly", "bilinear_sampler_3d", "coords_grid_3d",
           "upflow_3d", "flow_step", "make_corr_block", "resolve_precision", "pyramid_bytes", "hbm_available"]


_CANON = {ops.DVC_F32: "fp32", ops.DVC_BF16: "bf16", ops.DVC_F16: "fp16"}


def resolve_precision(fmap: torch.Tensor, precision: Optional[str]) -> str:
    """Storage/MFMA precision of the pyramid.  Explicit argument > DVCCORR_PRECISION >
    AMP policy > input dtype.

    AMP policy: the reference's Trainer runs RAFTDVC.forward under
    torch.amp.autocast('cuda') (trainer.py:249-252), so its CorrBlock matmul and
    avg_pool3d produce an fp16 pyramid (corr.py:155-167) even though the fmaps are
    cast to float32 first (raft_dvc.py:366-367), while grid_sample autocasts back to
    float32.  Inside an enabled CUDA autocast region (the float16 one: the reference's
    trainer uses autocast's default dtype) this block likewise packs, builds and stores
    fp16 (v_mfma_f32_32x32x16_f16) and returns float32 lookups; an autocast region set to
    bfloat16 gives bf16.  Outside autocast, float32 fmaps build in exact f32.  The on-the-fly
    block follows the same policy: under autocast its window dots run on fp16 MFMA
    (v_mfma_f32_16x16x32_f16), as the reference's CorrBlockOnTheFly einsum runs in fp16
    (corr_otf.py:198-237)."""
    if precision is None:
        precision = os.environ.get("DVCCORR_PRECISION") or None
    if precision is None and fmap.is_cuda and torch.is_autocast_enabled("cuda"):
        precision = "bf16" if torch.get_autocast_dtype("cuda") == torch.bfloat16 else "fp16"
    if precision is None:
        precision = {torch.float32: "fp32", torch.float16: "fp16"}.get(fmap.dtype, "bf16")
    return _CANON[ops.dtype_code(precision)]


def _wants_grad(*ts: torch.Tensor) -> bool:
    return torch.is_grad_enabled() and any(t.requires_grad for t in ts)


def _check_backward_support(lay, C: int, radius: int, legacy: bool) -> None:
    """Raise at construction (not after twelve forward lookups) when dvc_corr_backward cannot
    differentiate this block (include/dvccorr.h: radius 1..6; any C -- the gradient kernels run per
    128-channel group, as the reference's CUDA backward is templated for C in {16, 64, 128, 256},
    corr_otf_cuda.cu:537-541)."""
    if not 1 <= radius <= 6:
        raise NotImplementedError(f"dvccorr backward supports radius 1..6, got {radius}")


def pyramid_bytes(B: int, C: int, H: int, W: int, D: int, num_levels: int, precision: str = "fp32") -> int:
    """HBM bytes of the materialised pyramid CorrBlock allocates (B x N rows of row_stride values)."""
    lay = layout(H, W, D, num_levels, C)
    esz = 4 if precision == "fp32" else 2
    return B * H * W * D * lay.row_stride * esz + 2 * ops.GUARD_BYTES


def hbm_available(device) -> int:
    """Bytes a new allocation can get: free device memory plus the caching allocator's unused reserve."""
    device = torch.device(device)
    free, _total = torch.cuda.mem_get_info(device)
    return int(free + torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device))


class _Block:
    """Shared __call__: coords check, then the dvccorr operators (lookup_ad when grad is needed)."""

    def _check_coords(self, coords: torch.Tensor) -> None:
        B, _, H, W, D = self.shape
        if coords.ndim != 5 or tuple(coords.shape) != (B, 3, H, W, D):
            raise ValueError(f"coords must be (B, 3, H, W, D) = {(B, 3, H, W, D)}; got {tuple(coords.shape)}")

    def _convc1_fusable(self, weight: torch.Tensor, bias: torch.Tensor, w: torch.Tensor) -> bool:
        """The fused convc1 kernels cover radius 1..4, 96 output channels and no legacy level with W != D: a bf16 /
        fp16 block with fp16 MFMA operands, and (round 5, materialised blocks only) an fp32 block through the exact
        split consumer (bf16 hi/lo operands, fp32 tolerance; the reference's fp32 evaluation path,
        evaluate_phase1.py:115-131).  The on-the-fly fp32 block keeps the composition.  With gradients (the
        Trainer's path, trainer.py:249-257) the fused kernel runs as dvccorr::lookup_convc1_ad (_convc1_grad)."""
        return ((self.precision in ("bf16", "fp16") or (self.precision == "fp32" and isinstance(self, CorrBlock)))
                and 1 <= self.radius <= ops._lib.PROJ_MAX_RADIUS and w.shape[0] == ops._lib.PROJ_COUT
                and not (self.legacy_wd_swap and any(lw != ld and min(lh, lw, ld) > 1
                                                     for lh, lw, ld in self._lay.levels())))

    def _convc1_grad(self, weight: torch.Tensor, bias: torch.Tensor) -> bool:
        return torch.is_grad_enabled() and (weight.requires_grad or bias.requires_grad or
                                            self._grad_fmaps is not None)

    def _convc1_ad(self, coords: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, packed: torch.Tensor,
                   corr: Optional[torch.Tensor]) -> torch.Tensor:
        """relu(convc1(lookup)) through dvccorr::lookup_convc1_ad: the fused kernel forward, gradients for the
        fmaps (when the block's fmaps require grad), convc1.weight and convc1.bias."""
        B, C, H, W, D = self.shape
        f1, f2 = self._grad_fmaps if self._grad_fmaps is not None else (coords.new_empty(0), coords.new_empty(0))
        out = library.lookup_convc1_ad(f1, f2, weight, bias, corr, self._q, self._t, coords.reshape(B, 3, H * W * D),
                                       packed, C, H, W, D, self.num_levels, self.radius, self.legacy_wd_swap,
                                       self._dt, getattr(self, "_ldt", self._dt))
        return out.view(B, -1, H, W, D)

    def _convc1_composition(self, coords: torch.Tensor, w: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        out = self(coords)
        return torch.relu(torch.nn.functional.conv3d(out, w.reshape(w.shape[0], -1, 1, 1, 1), bias))

    def __call__(self, coords: torch.Tensor) -> torch.Tensor:
        self._check_coords(coords)
        B, C, H, W, D = self.shape
        flat = coords.reshape(B, 3, H * W * D)
        if self._grad_fmaps is not None and torch.is_grad_enabled():
            out = library.lookup_ad(*self._grad_fmaps, getattr(self, "_corr", None), self._q, self._t, flat, C, H,
                                    W, D, self.num_levels, self.radius, self.legacy_wd_swap, self._dt)
        else:
            out = self._lookup_flat(flat)
        return out.view(B, -1, H, W, D)


def brick_flag(lay, radius: int, legacy: bool, eligible: bool, bricked: Optional[bool] = None) -> int:
    """DVC_BRICKED when the materialised pyramid should store its wide levels in (1, 8, 8) bricks: a GEMM-built
    inference pyramid (the pooled build and the backward read the linear layout) whose lookups run on the tile
    kernel (radius 1..6, <= 4 levels, no legacy W != D bricked level).  bricked=False forces the linear layout
    (e.g. to A/B the walk kernels); DVCCORR_BRICKED=0 turns the default off."""
    if bricked is False or not eligible or os.environ.get("DVCCORR_BRICKED", "1") == "0":
        return 0
    if not (1 <= radius <= 6) or lay.num_levels > 4:
        return 0
    m = ops.bricked_levels(lay)
    if m == 0 or (legacy and any((m >> l) & 1 and lay.W[l] != lay.D[l] for l in range(lay.num_levels))):
        return 0
    return ops.DVC_BRICKED


def brick_index(h: int, w: int, dp: int, device) -> torch.Tensor:
    """Brick slot of each level voxel in (y, x, z) order: ((y w/8 + x/8) dp/8 + z/8) 64 + (x%8) 8 + z%8."""
    y, x, z = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device),
                             torch.arange(dp, device=device), indexing="ij")
    return ((((y * (w // 8)) + x // 8) * (dp // 8) + z // 8) * 64 + (x % 8) * 8 + z % 8).reshape(-1)


def _check_fmaps(fmap1: torch.Tensor, fmap2: torch.Tensor) -> None:
    if fmap1.ndim != 5:
        raise ValueError(f"Expected 5D feature maps (B, C, H, W, D); got {fmap1.ndim}D")
    if fmap1.shape != fmap2.shape:
        raise ValueError(f"fmap1 and fmap2 must have matching shapes; got {tuple(fmap1.shape)} vs "
                         f"{tuple(fmap2.shape)}")


class CorrBlock(_Block):
    """All-pairs 3-D correlation pyramid + radius-r trilinear lookup (materialised).

    Gradient precision (dvc_corr_backward, include/dvccorr.h): bf16 / fp16 blocks sum the gradients on the matrix
    cores from 16-bit window gradients (the one fp16 rounding of d(corr) the reference's AMP backward applies,
    trainer.py:249-257).  fp32 blocks run the same kernels on bf16 hi/lo splits of every operand, ~2^-16 relative
    per product -- not the exact fp32 sums of the reference's autograd: the golden gradients agree to <= 1e-5
    (tests/test_gpu_backward.py, GRAD_TOL).  dvccorr._lib.set_tuning("bwd_mfma", 0) selects the exact fp32 VALU kernels
    (process-wide, so also for the backward that the autograd engine runs on its own thread)."""

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 legacy_wd_swap: bool = False, *, precision: Optional[str] = None, build: str = "gemm",
                 bricked: Optional[bool] = None):
        _check_fmaps(fmap1, fmap2)
        self.num_levels = num_levels
        self.radius = radius
        self.legacy_wd_swap = legacy_wd_swap
        B, C, H, W, D = fmap1.shape
        self.shape = (B, C, H, W, D)
        self._lay = layout(H, W, D, num_levels, C)      # RuntimeError where avg_pool3d would raise
        self.precision = resolve_precision(fmap1, precision)
        self._dt = ops.dtype_code(self.precision)
        self._grad_fmaps = (fmap1, fmap2) if _wants_grad(fmap1, fmap2) else None
        if self._grad_fmaps is not None:
            _check_backward_support(self._lay, C, radius, legacy_wd_swap)
        if build not in ("gemm", "pool"):
            raise ValueError(f"build must be 'gemm' or 'pool', got {build!r}")
        ops._need_cuda(fmap1, fmap2)
        need = pyramid_bytes(B, C, H, W, D, num_levels, self.precision)
        avail = hbm_available(fmap1.device)
        if need > avail:
            raise torch.cuda.OutOfMemoryError(
                f"dvccorr.CorrBlock: the materialised {self.precision} pyramid of ({H},{W},{D}) x {num_levels} levels "
                f"needs {need / 2**30:.1f} GiB, {avail / 2**30:.1f} GiB of HBM is available; use "
                f"CorrBlockFused (corr_impl 'mi355x_fused' / 'mi355x_auto'), which never materialises it")
        # levels with >= 64-byte z-rows in (1, 8, 8) bricks (DVC_BRICKED): fewer HBM lines per lookup window
        self._brick = brick_flag(self._lay, radius, legacy_wd_swap, build == "gemm" and self._grad_fmaps is None,
                                 bricked)
        self._ldt = self._dt | self._brick              # the lookups' store dtype code (with the layout flag)
        q = ops.pack_queries(fmap1.detach().reshape(B, C, H * W * D), self._dt)
        t = ops.pack_targets(fmap2.detach(), num_levels, self._ldt)
        # the backward needs the packed operands (O(C * voxels)): keep them only then
        self._q, self._t = (q, t) if self._grad_fmaps is not None else (None, None)
        if build == "gemm":       # every level from the pooled targets, one launch
            self._corr = library.build(q, t, C, H, W, D, num_levels, self._dt)
        elif build == "pool":     # the reference's op order: level 0 GEMM, then avg-pool the volume
            corr = ops.alloc_corr(B, H * W * D, self._lay.row_stride, self._dt, q.device, zero=True)
            ops.build(q, t, C, H, W, D, num_levels, self._dt, self._dt, 0, self._lay.level_elems[0], out=corr)
            for l in range(num_levels - 1):
                ops.pool(corr, H, W, D, num_levels, l, self._dt)
            self._corr = corr

    @property
    def corr_pyramid(self) -> List[torch.Tensor]:
        """The pyramid shaped like the reference's list: (B*N, 1, H_l, W_l, D_l) per level -- zero-copy views,
        except for bricked levels (DVC_BRICKED), which are gathered back into (h, w, d) order."""
        B, _, H, W, D = self.shape
        flat = self._corr.reshape(B * H * W * D, self._lay.row_stride)
        mask = ops.bricked_levels(self._lay) if self._brick else 0
        views = []
        for l, (h, w, d) in enumerate(self._lay.levels()):
            dp = self._lay.Dp[l]
            off = self._lay.offset[l]
            sec = flat[:, off:off + h * w * dp]
            if (mask >> l) & 1:
                sec = sec[:, brick_index(h, w, dp, flat.device)]
            views.append(sec.reshape(B * H * W * D, 1, h, w, dp)[..., :d])
        return views

    def _lookup_flat(self, coords_flat: torch.Tensor) -> torch.Tensor:
        _, _, H, W, D = self.shape
        return library.lookup(self._corr, coords_flat, H, W, D, self.num_levels, self.radius, self.legacy_wd_swap,
                              self._ldt)

    def lookup_convc1(self, coords: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        """F.relu(convc1(self(coords))) -> (B, 96, H, W, D) fp32 with convc1 fused into the lookup.

        The motion encoder's first layer (update.py:219-222, 246: Conv3d(L*(2r+1)^3, 96, 1) + ReLU)
        runs on fp16 MFMA (fp32 accumulation; the reference's AMP convc1 is fp16 too) inside the
        lookup kernel of a bf16 / fp16 block, so the L*(2r+1)^3-channel tensor never reaches HBM
        (dvc_corr_lookup_proj; tolerance 1e-2 max-normalised); an fp32 block splits both operands into
        bf16 hi + lo (three MFMAs per step, tolerance 1e-5).  Under autograd (fmaps, weight or bias
        requiring grad) it runs as dvccorr::lookup_convc1_ad, whose backward recomputes the lookup.
        Radii / conventions the fused kernel does not cover take the composition
        F.relu(F.conv3d(self(coords), weight, bias)) on the GPU."""
        self._check_coords(coords)
        B, _, H, W, D = self.shape
        w = weight.reshape(weight.shape[0], -1)
        if not self._convc1_fusable(weight, bias, w):
            return self._convc1_composition(coords, w, bias)
        packed = ops.proj_pack_cached(weight, self.num_levels, self.radius, self.legacy_wd_swap,
                                      exact=self.precision == "fp32")
        if self._convc1_grad(weight, bias):
            return self._convc1_ad(coords, weight, bias, packed, self._corr)
        out = ops.lookup_proj(self._corr, coords.reshape(B, 3, H * W * D), packed, bias, H, W, D,
                              self.num_levels, self.radius, self.legacy_wd_swap, self._ldt)
        return out.view(B, -1, H, W, D)


class CorrBlockFused(_Block):
    """On-the-fly lookup (no correlation volume), any sampler convention.

    Keeps the packed fmap1 rows and the packed fmap2 pyramid (O(C * voxels));
    each call computes the (2r+2)^3 window dots per query and interpolates them.
    """

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 legacy_wd_swap: bool = False, *, precision: Optional[str] = None):
        _check_fmaps(fmap1, fmap2)
        self.num_levels = num_levels
        self.radius = radius
        self.legacy_wd_swap = legacy_wd_swap
        B, C, H, W, D = fmap1.shape
        self.shape = (B, C, H, W, D)
        self._lay = layout(H, W, D, num_levels, C)
        self.precision = resolve_precision(fmap1, precision)
        self._dt = ops.dtype_code(self.precision)
        self._grad_fmaps = (fmap1, fmap2) if _wants_grad(fmap1, fmap2) else None
        if self._grad_fmaps is not None:
            _check_backward_support(self._lay, C, radius, legacy_wd_swap)
        self._q = ops.pack_queries(fmap1.detach().reshape(B, C, H * W * D), self._dt)
        self._t = ops.pack_targets(fmap2.detach(), num_levels, self._dt)

    def _lookup_flat(self, coords_flat: torch.Tensor) -> torch.Tensor:
        _, C, H, W, D = self.shape
        return library.lookup_fused(self._q, self._t, coords_flat, C, H, W, D, self.num_levels, self.radius,
                                    self.legacy_wd_swap, self._dt)

    def lookup_convc1(self, coords: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        """F.relu(convc1(self(coords))) -> (B, 96, H, W, D) fp32 with convc1 fused into the on-the-fly lookup
        (dvc_corr_lookup_fused_proj): the L*(2r+1)^3 channels never reach HBM, and the queries are grouped by
        window position so each workgroup's window union is small.  Same numerics and fallbacks as
        CorrBlock.lookup_convc1 (fp16 convc1 operands, tolerance 1e-2; fp32 blocks, gradients, radii > 4,
        legacy W != D levels and C_pad outside {32, 64, 128} take relu(conv3d(self(coords))))."""
        self._check_coords(coords)
        B, C, H, W, D = self.shape
        w = weight.reshape(weight.shape[0], -1)
        if not (self._convc1_fusable(weight, bias, w) and self._lay.c_pad in (32, 64, 128)):
            return self._convc1_composition(coords, w, bias)
        packed = ops.proj_pack_cached(weight, self.num_levels, self.radius, self.legacy_wd_swap)
        if self._convc1_grad(weight, bias):
            return self._convc1_ad(coords, weight, bias, packed, None)
        out = library.lookup_fused_proj(self._q, self._t, coords.reshape(B, 3, H * W * D), packed, bias, C, H, W,
                                        D, self.num_levels, self.radius, self.legacy_wd_swap, self._dt)
        return out.view(B, -1, H, W, D)


class CorrBlockOnTheFly(CorrBlockFused):
    """Reference-signature on-the-fly block (corr_otf.py:51-94).

    Like the reference it implements the LEGACY sampler convention
    (corr_otf.py:227-234); chunk_size / use_checkpoint only shape the
    reference's PyTorch memory use and are validated and ignored here.
    """

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 chunk_size: int = 27, use_checkpoint: bool = True, *, precision: Optional[str] = None):
        if fmap1.shape != fmap2.shape:
            raise ValueError(f"fmap1 and fmap2 must have matching shapes; got {tuple(fmap1.shape)} vs "
                             f"{tuple(fmap2.shape)}")
        if fmap1.ndim != 5:
            raise ValueError(f"Expected 5D feature maps (B, C, H, W, D); got {fmap1.ndim}D")
        if chunk_size < 1:
            raise ValueError(f"chunk_size must be >= 1; got {chunk_size}")
        self.chunk_size = chunk_size
        self.use_checkpoint = use_checkpoint
        super().__init__(fmap1, fmap2, num_levels, radius, legacy_wd_swap=True, precision=precision)


def bilinear_sampler_3d(vol: torch.Tensor, coords: torch.Tensor, legacy_wd_swap: bool = False) -> torch.Tensor:
    """vol (B, C, H, W, D), coords (B, H', W', D', 3) in (h, w, d) -> (B, C, H', W', D').

    Forward only (k_sample3d): the reference uses it inside CorrBlock, which this package
    differentiates as a whole; a standalone call on inputs that require grad raises instead of
    silently returning a tensor with no autograd history."""
    if vol.ndim != 5 or coords.ndim != 5 or coords.shape[-1] != 3 or coords.shape[0] != vol.shape[0]:
        raise ValueError(f"bad shapes vol {tuple(vol.shape)} coords {tuple(coords.shape)}")
    if _wants_grad(vol, coords):
        raise NotImplementedError("dvccorr.bilinear_sampler_3d has no backward; call it under torch.no_grad() "
                                  "or use the reference's F.grid_sample path for gradients")
    B, C = vol.shape[:2]
    out = ops.sample3d(vol, coords.reshape(B, -1, 3), legacy_wd_swap)
    return out.view(B, C, *coords.shape[1:4])


def coords_grid_3d(batch: int, ht: int, wd: int, dp: int, device: torch.device) -> torch.Tensor:
    """Identity grid (B, 3, H, W, D), channel c = index along axis c (h, w, d).

    On the GPU this is k_coords_grid (dvc_coords_grid); a CPU device (input
    generation in tests and bench) builds the same integers with torch.
    """
    if torch.device(device).type == "cuda":
        return ops.coords_grid(batch, ht, wd, dp, device)
    axes = [torch.arange(s, device=device, dtype=torch.float32) for s in (ht, wd, dp)]
    grid = torch.stack(torch.meshgrid(*axes, indexing="ij"), dim=0)
    return grid.unsqueeze(0).expand(batch, 3, ht, wd, dp).contiguous()


def _upflow_adjoint(grad_up: torch.Tensor, lo_shape) -> torch.Tensor:
    """Adjoint of upflow_3d: the per-axis scale of channels 0..2 (corr.py:242-251), then the
    transpose of trilinear align_corners=True interpolation (ATen's upsample_trilinear3d_backward,
    the op autograd runs for the reference's F.interpolate at corr.py:234-239)."""
    B, C, h, w, d = lo_shape
    H, W, D = grad_up.shape[2:]
    g = grad_up.float().clone()
    for c, s in enumerate((H / h, W / w, D / d)[:min(C, 3)]):
        g[:, c] *= s
    return torch.ops.aten.upsample_trilinear3d_backward(g, [H, W, D], [B, C, h, w, d], True, None, None, None)


class _UpflowFn(torch.autograd.Function):
    """upflow_3d with the reference's gradient (flow_predictions carry the loss back to delta_flow
    and the update block, raft_dvc.py:482-486): forward k_upflow, backward its adjoint."""

    @staticmethod
    def forward(ctx, flow, target_shape):
        ctx.lo_shape = tuple(flow.shape)
        ctx.in_dtype = flow.dtype
        return ops.upflow(flow, target_shape)

    @staticmethod
    def backward(ctx, grad_up):
        return _upflow_adjoint(grad_up, ctx.lo_shape).to(ctx.in_dtype), None


class _FlowStepFn(torch.autograd.Function):
    """flow_step with gradients: d coords1 = d delta = d coords1' + adjoint(d flow_up)
    (coords1' = coords1 + delta_flow, flow_up = upflow_3d(coords1' - coords0))."""

    @staticmethod
    def forward(ctx, coords1, delta_flow, target_shape):
        ctx.lo_shape = tuple(coords1.shape)
        ctx.dtypes = (coords1.dtype, None if delta_flow is None else delta_flow.dtype)
        return ops.flow_step(coords1, delta_flow, target_shape)

    @staticmethod
    def backward(ctx, g_coords, g_up):
        g = torch.zeros(ctx.lo_shape, dtype=torch.float32, device=(g_up if g_up is not None else g_coords).device)
        if g_coords is not None:
            g = g + g_coords.float()
        if g_up is not None:
            g = g + _upflow_adjoint(g_up, ctx.lo_shape)
        d1 = g.to(ctx.dtypes[0]) if ctx.needs_input_grad[0] else None
        d2 = g.to(ctx.dtypes[1]) if ctx.needs_input_grad[1] else None
        return d1, d2, None


def upflow_3d(flow: torch.Tensor, target_shape=None, scale_factor: int = 8) -> torch.Tensor:
    """upflow_3d (src/core/corr.py:211-253): trilinear, align_corners=True, channels 0..2
    scaled by target/source size per axis -- one k_upflow pass (dvc_upflow).  Differentiable."""
    if target_shape is None:
        _, _, h, w, d = flow.shape
        target_shape = (h * scale_factor, w * scale_factor, d * scale_factor)
    target_shape = tuple(int(v) for v in target_shape)
    if _wants_grad(flow):
        return _UpflowFn.apply(flow, target_shape)
    return ops.upflow(flow, target_shape)


def flow_step(coords1: torch.Tensor, delta_flow: Optional[torch.Tensor], target_shape):
    """RAFTDVC.forward's per-iteration tail (raft_dvc.py:482-485) in one k_upflow pass:

        coords1 = coords1 + delta_flow
        flow_up = upflow_3d(coords1 - coords0, target_shape=target_shape)

    coords0 is the identity grid (raft_dvc.py:293), formed in registers.  Returns
    (coords1, flow_up); the input coords1 is not modified.  Differentiable w.r.t.
    coords1 and delta_flow (the flow loss reaches the update block through flow_up).
    """
    target_shape = tuple(int(v) for v in target_shape)
    if _wants_grad(coords1, *(() if delta_flow is None else (delta_flow,))):
        return _FlowStepFn.apply(coords1, delta_flow, target_shape)
    return ops.flow_step(coords1, delta_flow, target_shape)


# CorrBlock keywords with no meaning for the on-the-fly block (no pyramid is stored)
_MATERIALISED_ONLY_KW = ("build", "bricked")


def make_corr_block(impl: str, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                    sampler_version: int = 2, **kw):
    """The dispatch RAFTDVC.forward performs on config.corr_impl (raft_dvc.py:369-420), for the new impls.

    impl "mi355x"        -> CorrBlock (materialised pyramid, fixed or legacy convention)
    impl "mi355x_fused"  -> CorrBlockFused (on-the-fly, fixed or legacy convention)
    impl "mi355x_auto"   -> CorrBlock when its pyramid fits the free HBM (with 10 % headroom for the
                            rest of the step), else CorrBlockFused (failure detection)
    """
    if sampler_version not in (1, 2):
        raise ValueError(f"Invalid corr_sampler_version: {sampler_version!r}. Must be 1 (legacy W<->D-swapped) "
                         f"or 2 (fixed).")
    legacy = sampler_version == 1
    if impl == "mi355x":
        return CorrBlock(fmap1, fmap2, num_levels, radius, legacy_wd_swap=legacy, **kw)
    if impl == "mi355x_fused":
        return CorrBlockFused(fmap1, fmap2, num_levels, radius, legacy_wd_swap=legacy, **kw)
    if impl == "mi355x_auto":
        _check_fmaps(fmap1, fmap2)
        B, C, H, W, D = fmap1.shape
        prec = resolve_precision(fmap1, kw.get("precision"))
        fits = pyramid_bytes(B, C, H, W, D, num_levels, prec) <= 0.9 * hbm_available(fmap1.device)
        cls = CorrBlock if fits else CorrBlockFused
        kw = {k: v for k, v in kw.items() if cls is CorrBlock or k not in _MATERIALISED_ONLY_KW}
        return cls(fmap1, fmap2, num_levels, radius, legacy_wd_swap=legacy, **kw)
    raise ValueError(f"Invalid corr_impl for dvccorr: {impl!r}. Must be 'mi355x', 'mi355x_fused' or 'mi355x_auto'")
