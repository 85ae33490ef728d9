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
bf16 MFMA and stores bf16 (tolerance 1e-2), halving the HBM traffic; the
default follows the input dtype (fp16/bf16 inputs -> bf16), overridable with
the DVCCORR_PRECISION environment variable.

Backward: when a feature map requires grad, every call is an autograd node whose
backward runs dvc_corr_backward (sparse per-query window gradients, no dense
d(corr), no atomics) and returns d fmap1 / d fmap2; coordinates get no gradient,
as RAFTDVC.forward detaches them (raft_dvc.py:441).  Twelve calls on one block
accumulate in autograd like the reference's twelve grid_sample calls.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from . import ops
from ._lib import layout

__all__ = ["CorrBlock", "CorrBlockFused", "CorrBlockOnTheFly", "bilinear_sampler_3d", "coords_grid_3d",
           "upflow_3d", "flow_step", "make_corr_block", "resolve_precision"]


def resolve_precision(fmap: torch.Tensor, precision: Optional[str]) -> str:
    """Storage/MFMA precision of the pyramid.  Explicit argument > DVCCORR_PRECISION >
    AMP policy > input dtype.

    AMP policy: the reference's Trainer runs RAFTDVC.forward under
    torch.amp.autocast('cuda') (trainer.py:249-252), so its CorrBlock matmul and
    avg_pool3d produce an fp16 pyramid (corr.py:155-167) even though the fmaps are
    cast to float32 first (raft_dvc.py:366-367), while grid_sample autocasts back to
    float32.  Inside an enabled CUDA autocast region this block likewise builds and
    stores 16-bit (bf16: same 2 bytes per value, fp32 range) and returns float32
    lookups; outside it, float32 fmaps build in exact f32."""
    if precision is None:
        precision = os.environ.get("DVCCORR_PRECISION") or None
    if precision is None and fmap.is_cuda and torch.is_autocast_enabled("cuda"):
        precision = "bf16"
    if precision is None:
        precision = "fp32" if fmap.dtype == torch.float32 else "bf16"
    ops.dtype_code(precision)
    return "bf16" if precision in ("bf16", "bfloat16") else "fp32"


def _wants_grad(*ts: torch.Tensor) -> bool:
    return torch.is_grad_enabled() and any(t.requires_grad for t in ts)


class _LookupFn(torch.autograd.Function):
    """One lookup call as an autograd node (reference: autograd through corr.py:141-208).

    forward: the block's lookup kernels; backward: dvc_corr_backward -> (d fmap1, d fmap2).
    Coordinates get no gradient (RAFTDVC.forward detaches them, raft_dvc.py:441)."""

    @staticmethod
    def forward(ctx, coords, fmap1, fmap2, blk):
        ctx.blk = blk
        ctx.legacy = blk.legacy_wd_swap
        ctx.dtypes = (fmap1.dtype, fmap2.dtype)
        ctx.save_for_backward(coords)
        return blk._lookup(coords)

    @staticmethod
    def backward(ctx, grad_out):
        (coords,) = ctx.saved_tensors
        blk = ctx.blk
        B, C, H, W, D = blk.shape
        N = H * W * D
        d1, d2 = ops.corr_backward(blk._q, blk._t, coords.reshape(B, 3, N), grad_out.reshape(B, -1, N), C, H, W, D,
                                   blk.num_levels, blk.radius, ctx.legacy, blk._dt)
        return None, d1.view(B, C, H, W, D).to(ctx.dtypes[0]), d2.to(ctx.dtypes[1]), None


class _Block:
    """Shared __call__: coords check, then the kernels (wrapped in _LookupFn when grad is needed)."""

    def _check_coords(self, coords: torch.Tensor) -> None:
        B, _, H, W, D = self.shape
        if coords.ndim != 5 or tuple(coords.shape) != (B, 3, H, W, D):
            raise ValueError(f"coords must be (B, 3, H, W, D) = {(B, 3, H, W, D)}; got {tuple(coords.shape)}")

    def __call__(self, coords: torch.Tensor) -> torch.Tensor:
        self._check_coords(coords)
        if self._grad_fmaps is not None and torch.is_grad_enabled():
            return _LookupFn.apply(coords, *self._grad_fmaps, self)
        return self._lookup(coords)


def _check_fmaps(fmap1: torch.Tensor, fmap2: torch.Tensor) -> None:
    if fmap1.ndim != 5:
        raise ValueError(f"Expected 5D feature maps (B, C, H, W, D); got {fmap1.ndim}D")
    if fmap1.shape != fmap2.shape:
        raise ValueError(f"fmap1 and fmap2 must have matching shapes; got {tuple(fmap1.shape)} vs "
                         f"{tuple(fmap2.shape)}")


class CorrBlock(_Block):
    """All-pairs 3-D correlation pyramid + radius-r trilinear lookup (materialised)."""

    def __init__(self, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                 legacy_wd_swap: bool = False, *, precision: Optional[str] = None, build: str = "gemm"):
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
        q = ops.pack_queries(fmap1.detach().reshape(B, C, H * W * D), self._dt)
        t = ops.pack_targets(fmap2.detach(), num_levels, self._dt)
        # the backward needs the packed operands (O(C * voxels)): keep them only then
        self._q, self._t = (q, t) if self._grad_fmaps is not None else (None, None)
        if build == "gemm":       # every level from the pooled targets, one launch
            self._corr = ops.build(q, t, C, H, W, D, num_levels, self._dt, self._dt)
        elif build == "pool":     # the reference's op order: level 0 GEMM, then avg-pool the volume
            corr = ops.alloc_corr(B, H * W * D, self._lay.row_stride, self._dt, q.device, zero=True)
            ops.build(q, t, C, H, W, D, num_levels, self._dt, self._dt, 0, self._lay.level_elems[0], out=corr)
            for l in range(num_levels - 1):
                ops.pool(corr, H, W, D, num_levels, l, self._dt)
            self._corr = corr
        else:
            raise ValueError(f"build must be 'gemm' or 'pool', got {build!r}")

    @property
    def corr_pyramid(self) -> List[torch.Tensor]:
        """Zero-copy views shaped like the reference's list: (B*N, 1, H_l, W_l, D_l) per level."""
        B, _, H, W, D = self.shape
        flat = self._corr.reshape(B * H * W * D, self._lay.row_stride)
        views = []
        for l, (h, w, d) in enumerate(self._lay.levels()):
            dp = self._lay.Dp[l]
            off = self._lay.offset[l]
            v = flat[:, off:off + h * w * dp].reshape(B * H * W * D, 1, h, w, dp)[..., :d]
            views.append(v)
        return views

    def _lookup(self, coords: torch.Tensor) -> torch.Tensor:
        B, _, H, W, D = self.shape
        out = ops.lookup(self._corr, coords.reshape(B, 3, H * W * D), H, W, D, self.num_levels, self.radius,
                         self.legacy_wd_swap, self._dt)
        return out.view(B, -1, H, W, D)

    def lookup_convc1(self, coords: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        """F.relu(convc1(self(coords))) -> (B, 96, H, W, D) fp32 with convc1 fused into the lookup.

        The motion encoder's first layer (update.py:219-222, 246: Conv3d(L*(2r+1)^3, 96, 1) + ReLU)
        runs on bf16 MFMA inside the lookup kernel, so the L*(2r+1)^3-channel tensor never reaches
        HBM (dvc_corr_lookup_proj; tolerance 1e-2 max-normalised, bf16 operands, fp32 accumulation).
        When gradients are needed, or for radii/conventions the fused kernel does not cover, it is
        the unfused composition F.relu(F.conv3d(self(coords), weight, bias)) on the GPU."""
        self._check_coords(coords)
        B, _, H, W, D = self.shape
        w = weight.reshape(weight.shape[0], -1)
        fused_ok = (not (torch.is_grad_enabled() and (weight.requires_grad or bias.requires_grad or
                                                      self._grad_fmaps is not None))
                    and 1 <= self.radius <= ops._lib.PROJ_MAX_RADIUS and w.shape[0] == ops._lib.PROJ_COUT
                    and not (self.legacy_wd_swap and any(lw != ld and min(lh, lw, ld) > 1
                                                         for lh, lw, ld in self._lay.levels())))
        if not fused_ok:
            out = self(coords)
            return torch.relu(torch.nn.functional.conv3d(out, w.reshape(w.shape[0], -1, 1, 1, 1), bias))
        packed = ops.proj_pack_cached(weight, self.num_levels, self.radius, self.legacy_wd_swap)
        out = ops.lookup_proj(self._corr, coords.reshape(B, 3, H * W * D), packed, bias, H, W, D,
                              self.num_levels, self.radius, self.legacy_wd_swap, self._dt)
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
        self._q = ops.pack_queries(fmap1.detach().reshape(B, C, H * W * D), self._dt)
        self._t = ops.pack_targets(fmap2.detach(), num_levels, self._dt)
        self._ws = ops.fused_workspace(B, H * W * D, num_levels, radius, fmap1.device)

    def _lookup(self, coords: torch.Tensor) -> torch.Tensor:
        B, C, H, W, D = self.shape
        out = ops.lookup_fused(self._q, self._t, coords.reshape(B, 3, H * W * D), C, H, W, D, self.num_levels,
                               self.radius, self.legacy_wd_swap, self._dt, workspace=self._ws)
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
    """vol (B, C, H, W, D), coords (B, H', W', D', 3) in (h, w, d) -> (B, C, H', W', D')."""
    if vol.ndim != 5 or coords.ndim != 5 or coords.shape[-1] != 3 or coords.shape[0] != vol.shape[0]:
        raise ValueError(f"bad shapes vol {tuple(vol.shape)} coords {tuple(coords.shape)}")
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


def upflow_3d(flow: torch.Tensor, target_shape=None, scale_factor: int = 8) -> torch.Tensor:
    """upflow_3d (src/core/corr.py:211-253): trilinear, align_corners=True, channels 0..2
    scaled by target/source size per axis -- one k_upflow pass (dvc_upflow)."""
    if target_shape is None:
        _, _, h, w, d = flow.shape
        target_shape = (h * scale_factor, w * scale_factor, d * scale_factor)
    return ops.upflow(flow, target_shape)


def flow_step(coords1: torch.Tensor, delta_flow: Optional[torch.Tensor], target_shape):
    """RAFTDVC.forward's per-iteration tail (raft_dvc.py:482-485) in one k_upflow pass:

        coords1 = coords1 + delta_flow
        flow_up = upflow_3d(coords1 - coords0, target_shape=target_shape)

    coords0 is the identity grid (raft_dvc.py:293), formed in registers.  Returns
    (coords1, flow_up); the input coords1 is not modified.
    """
    return ops.flow_step(coords1, delta_flow, target_shape)


def make_corr_block(impl: str, fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4, radius: int = 4,
                    sampler_version: int = 2, **kw):
    """The dispatch RAFTDVC.forward performs on config.corr_impl (raft_dvc.py:369-420), for the new impls.

    impl "mi355x"        -> CorrBlock (materialised pyramid, fixed or legacy convention)
    impl "mi355x_fused"  -> CorrBlockFused (on-the-fly, fixed or legacy convention)
    """
    if sampler_version not in (1, 2):
        raise ValueError(f"Invalid corr_sampler_version: {sampler_version!r}. Must be 1 (legacy W<->D-swapped) "
                         f"or 2 (fixed).")
    legacy = sampler_version == 1
    if impl == "mi355x":
        return CorrBlock(fmap1, fmap2, num_levels, radius, legacy_wd_swap=legacy, **kw)
    if impl == "mi355x_fused":
        return CorrBlockFused(fmap1, fmap2, num_levels, radius, legacy_wd_swap=legacy, **kw)
    raise ValueError(f"Invalid corr_impl for dvccorr: {impl!r}. Must be 'mi355x' or 'mi355x_fused'")
