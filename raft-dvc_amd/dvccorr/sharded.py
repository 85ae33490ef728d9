"""Query-voxel sharding of the correlation block across the GPUs of one node.

Rows of the correlation volume are independent: row q of every pyramid level
depends only on fmap1[:, q] and all of fmap2, and the lookup of q only on
those rows and coords[q].  So each rank owns a contiguous
slab of H planes of the query volume:

  * fmap2 is replicated once per forward with one RCCL all-gather of the
    per-rank fmap2 slabs (each GPU receives (n-1)/n of fmap2 over its xGMI
    links in parallel);
  * each rank builds only its own rows of every level -- they never move
    (64^3 at 1/4: 19.6 GB/GPU bf16 at n=8 instead of 157 GB);
  * each lookup is shard-resident; gather_output=True additionally
    all-gathers the lookup output for an unsharded consumer.

Sharded results are bitwise equal to the single-GPU ones: the same kernels
run on the same rows.  The reference has no distributed code; this is new
design.  The per-rank compute is a pluggable backend (default: the HIP
library) so the partitioning / collective logic is testable on CPU (gloo).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import ops
from ._lib import layout
from .corr_block import resolve_precision


def slab_bounds(H: int, world: int, rank: int):
    """Contiguous H-plane slab [h0, h1) of `rank` (sizes differ by at most one)."""
    base, rem = divmod(H, world)
    h0 = rank * base + min(rank, rem)
    return h0, h0 + base + (1 if rank < rem else 0)


LOCAL = "local"   # group sentinel: this rank alone (data-parallel replicas, no collective)


def _world(group) -> int:
    if group == LOCAL:
        return 1
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _rank(group) -> int:
    if group == LOCAL:
        return 0
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


def all_gather_slab(slab: torch.Tensor, H: int, group=None, dim: int = 2, buf: Optional[torch.Tensor] = None,
                    async_op: bool = False):
    """The collective half of gather_slabs: every rank's slab (zero-padded to ceil(H / world) along `dim`)
    into buf[world, ...].  One collective, chosen from the group's backend -- identical on every rank, so
    the ranks' collective sequences cannot diverge, and a failing collective raises on every rank.
    async_op=True returns the work handle (wait() orders the current stream after the gather) instead of
    the buffer."""
    world = _world(group)
    maxh = -(-H // world)
    pad = maxh - slab.shape[dim]
    if pad:
        shape = list(slab.shape)
        shape[dim] = pad
        slab = torch.cat([slab, slab.new_zeros(shape)], dim=dim)
    slab = slab.contiguous()
    if buf is None:
        buf = slab.new_empty((world,) + tuple(slab.shape))
    if world == 1:
        buf[0].copy_(slab)
        work = None
    elif dist.get_backend(group) == "nccl":    # RCCL: one all-gather into the contiguous buffer
        work = dist.all_gather_into_tensor(buf, slab, group=group, async_op=async_op)
    else:                                      # gloo (CPU tests): list form
        work = dist.all_gather(list(buf.unbind(0)), slab, group=group, async_op=async_op)
    if async_op:
        return work if work is not None else _Done()
    return buf


class _Done:
    """Work handle of a collective that completed synchronously (world size 1)."""

    def wait(self):
        return True


def assemble_slabs(buf: torch.Tensor, H: int, dim: int = 2) -> torch.Tensor:
    """The local half of gather_slabs: buf[world, ...] (padded slabs) -> the full tensor along `dim`."""
    world = buf.shape[0]
    parts = []
    for r in range(world):
        h0, h1 = slab_bounds(H, world, r)
        parts.append(buf[r].narrow(dim, 0, h1 - h0))
    return torch.cat(parts, dim=dim)


def gather_slabs(slab: torch.Tensor, H: int, group=None, dim: int = 2) -> torch.Tensor:
    """All-gather H-slabs (split along `dim`) into the full tensor.  One collective."""
    if _world(group) == 1:
        return slab
    return assemble_slabs(all_gather_slab(slab, H, group, dim), H, dim)


class HipRows:
    """Default backend: this rank's query rows against the full target pyramid on the GPU."""

    def __init__(self, q_flat: torch.Tensor, fmap2: Optional[torch.Tensor], num_levels: int, radius: int, legacy: bool,
                 precision: str, impl: str, q_offset: int = 0, gathered=None):
        # gathered = (all_gather_slab's receive buffer, H): the targets are packed straight from the slabs
        # (dvc_pack_targets_gathered) instead of from an assembled copy of fmap2; fmap2 is then unused
        if gathered is not None and num_levels > 4:    # (the gathered pack is the single-pass one)
            fmap2, gathered = assemble_slabs(*gathered), None
        if gathered is not None:
            _, B, C, _, W, D = gathered[0].shape
            H = gathered[1]
        else:
            B, C, H, W, D = fmap2.shape
        self.dims = (C, H, W, D)
        self.L, self.R, self.legacy, self.impl = num_levels, radius, legacy, impl
        self.dt = ops.dtype_code(precision)
        # materialised rows: wide levels in (1, 8, 8) bricks, read by the tile lookups (corr_block.brick_flag)
        from .corr_block import brick_flag
        lay = layout(H, W, D, num_levels, C)
        self.ldt = self.dt | (brick_flag(lay, radius, legacy, True) if impl == "materialised" else 0)
        # (one stream: the query pack on a forked side stream beside the target pack was slower, 0.394-0.396 vs
        # 0.373-0.375 ms per 8-way slab step, profiles/r05/r05_ab_pack_side.txt)
        self.q = ops.pack_queries(q_flat, self.dt)
        if gathered is not None:
            self.t = ops.pack_targets_gathered(gathered[0], H, num_levels, self.ldt)
        else:
            self.t = ops.pack_targets(fmap2, num_levels, self.ldt)
        if impl == "materialised":
            self.corr = ops.build(self.q, self.t, C, H, W, D, num_levels, self.dt, self.dt)
        elif impl == "fused":
            self.ws = ops.fused_workspace(B, q_flat.shape[2], num_levels, radius, q_flat.device)
        else:
            raise ValueError(f"impl must be 'materialised' or 'fused', got {impl!r}")

    def lookup(self, coords_flat: torch.Tensor) -> torch.Tensor:
        C, H, W, D = self.dims
        if self.impl == "materialised":
            return ops.lookup(self.corr, coords_flat, H, W, D, self.L, self.R, self.legacy, self.ldt)
        return ops.lookup_fused(self.q, self.t, coords_flat, C, H, W, D, self.L, self.R, self.legacy, self.dt,
                                workspace=self.ws)

    def lookup_convc1(self, coords_flat: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        """relu(convc1(lookup)) of this rank's rows, convc1 fused into the lookup kernel (materialised:
        dvc_corr_lookup_proj, fused: dvc_corr_lookup_fused_proj) for a bf16 block; an fp32 block, or shapes
        the fused kernels do not cover, take relu(W . lookup + b) in fp32."""
        C, H, W, D = self.dims
        w = weight.reshape(weight.shape[0], -1)
        generic = self.legacy and any(lw != ld and min(lh, lw, ld) > 1
                                      for lh, lw, ld in layout(H, W, D, self.L, C).levels())
        fusable = (self.dt in (ops.dtype_code("bf16"), ops.dtype_code("fp16")) and 1 <= self.R <= ops._lib.PROJ_MAX_RADIUS
                   and w.shape[0] == ops._lib.PROJ_COUT and not generic
                   and (self.impl == "materialised" or layout(H, W, D, self.L, C).c_pad in (32, 64, 128)))
        if not fusable:
            out = self.lookup(coords_flat)
            return torch.relu(torch.matmul(w.float(), out) + bias.float().view(1, -1, 1))
        packed = ops.proj_pack_cached(weight, self.L, self.R, self.legacy)
        if self.impl == "materialised":
            return ops.lookup_proj(self.corr, coords_flat, packed, bias, H, W, D, self.L, self.R, self.legacy,
                                   self.ldt)
        if getattr(self, "pws", None) is None:   # sort keys + [B][N][96] rows, reused across lookups
            B, _, N = coords_flat.shape
            self.pws = torch.empty((max(ops.lib().dvc_lookup_fused_proj_workspace_bytes(B, N), 256),),
                                   dtype=torch.uint8, device=coords_flat.device)
        return ops.lookup_fused_proj(self.q, self.t, coords_flat, packed, bias, C, H, W, D, self.L, self.R,
                                     self.legacy, self.dt, workspace=self.pws)


class ShardedCorrBlock:
    """CorrBlock over this rank's H-slab of query voxels (fmap1 / coords slabs, full fmap2 gathered).

    Args:
        fmap1_slab, fmap2_slab: (B, C, h1-h0, W, D), this rank's slab_bounds(H) planes.
        H: full H extent of the feature maps.
        gather_output: all-gather every lookup output to the full (B, L*n^3, H, W, D).
        backend: per-rank compute (default HipRows); see tests/test_sharded_gloo.py.
    """

    def __init__(self, fmap1_slab: torch.Tensor, fmap2_slab: torch.Tensor, H: int, num_levels: int = 4,
                 radius: int = 4, legacy_wd_swap: bool = False, *, precision: Optional[str] = None,
                 impl: str = "materialised", group=None, gather_output: bool = False, build_events=None,
                 backend=HipRows):
        if torch.is_grad_enabled() and (fmap1_slab.requires_grad or fmap2_slab.requires_grad):
            raise NotImplementedError("ShardedCorrBlock is forward-only (inference and benchmarking): its "
                                      "lookups have no autograd node; build it under torch.no_grad() or use "
                                      "CorrBlock per rank for training")
        if fmap1_slab.shape != fmap2_slab.shape or fmap1_slab.ndim != 5:
            raise ValueError(f"slabs must be matching 5-D tensors; got {tuple(fmap1_slab.shape)} vs "
                             f"{tuple(fmap2_slab.shape)}")
        self.group = group
        self.world, self.rank = _world(group), _rank(group)
        h0, h1 = slab_bounds(H, self.world, self.rank)
        B, C, Hs, W, D = fmap1_slab.shape
        if Hs != h1 - h0:
            raise ValueError(f"rank {self.rank} slab has {Hs} planes, slab_bounds gives {h1 - h0}")
        self.H, self.h0, self.h1 = H, h0, h1
        self.shape = (B, C, Hs, W, D)
        self.num_levels, self.radius, self.legacy_wd_swap = num_levels, radius, legacy_wd_swap
        self.gather_output = gather_output
        precision = resolve_precision(fmap1_slab, precision)
        stream = torch.cuda.current_stream(fmap1_slab.device) if fmap1_slab.is_cuda else None
        if build_events is not None and stream is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        q_flat = fmap1_slab.reshape(B, C, Hs * W * D)
        if backend is HipRows and self.world > 1 and fmap2_slab.is_cuda:
            # the one data-path collective per forward; the targets are packed from its receive buffer
            buf = all_gather_slab(fmap2_slab.float(), H, group)
            self.rows = HipRows(q_flat, None, num_levels, radius, legacy_wd_swap, precision, impl, q_offset=h0 * W * D,
                                gathered=(buf, H))
        else:
            fmap2 = gather_slabs(fmap2_slab, H, group)       # the one data-path collective per forward
            self.rows = backend(q_flat, fmap2, num_levels, radius, legacy_wd_swap, precision, impl,
                                q_offset=h0 * W * D)
        if build_events is not None and stream is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(stream)
            build_events.append((e0, e1))

    def __call__(self, coords_slab: torch.Tensor) -> torch.Tensor:
        B, C, Hs, W, D = self.shape
        if tuple(coords_slab.shape) != (B, 3, Hs, W, D):
            raise ValueError(f"coords slab must be {(B, 3, Hs, W, D)}; got {tuple(coords_slab.shape)}")
        out = self.rows.lookup(coords_slab.reshape(B, 3, Hs * W * D)).view(B, -1, Hs, W, D)
        if self.gather_output:
            out = gather_slabs(out, self.H, self.group)
        return out

    def lookup_convc1(self, coords_slab: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
        """relu(convc1(self(coords_slab))) -> (B, 96, h1-h0, W, D) (or the full H with gather_output): the
        motion encoder's first layer (update.py:222, 246) fused into the lookup; the gathered output is
        96 channels instead of L*(2r+1)^3."""
        B, C, Hs, W, D = self.shape
        if tuple(coords_slab.shape) != (B, 3, Hs, W, D):
            raise ValueError(f"coords slab must be {(B, 3, Hs, W, D)}; got {tuple(coords_slab.shape)}")
        out = self.rows.lookup_convc1(coords_slab.reshape(B, 3, Hs * W * D), weight, bias).view(B, -1, Hs, W, D)
        if self.gather_output:
            out = gather_slabs(out, self.H, self.group)
        return out
