"""torch.library registrations of the correlation ops.

The drop-in blocks (corr_block.py) call these, so the hot path is visible to
the PyTorch dispatcher as named operators with shape functions:

    dvccorr::build(q, t, ...)                    -> corr pyramid (B, Nq, row_stride)   corr.py:141-167
    dvccorr::lookup(corr, coords, ...)           -> (B, L*(2r+1)^3, Nq) f32            corr.py:169-208
    dvccorr::lookup_fused(q, t, coords, ...)     -> (B, L*(2r+1)^3, Nq) f32            corr_otf.py:96-237
    dvccorr::lookup_fused_proj(q, t, coords, w, b, ...) -> (B, 96, Nq) f32 = relu(convc1(lookup_fused))
                                                                                       + update.py:246
    dvccorr::corr_backward(q, t, coords, g, ...) -> (d fmap1 (B, C, Nq), d fmap2)      autograd of corr.py:141-208
    dvccorr::lookup_convc1_ad(fmap1, fmap2, weight, bias, corr?, q, t, coords, packed_w, ...)
        relu(convc1(lookup)) differentiable (update.py:246): the fused kernel forward, the backward
        recomputes the lookup and feeds W^T (dy * relu') to dvccorr::corr_backward
    dvccorr::lookup_ad(fmap1, fmap2, corr?, q, t, coords, ...)
        the lookup as a differentiable op: fmap1 / fmap2 are its gradient carriers
        (the values it reads are the packed q / t / corr built from them), and the
        registered autograd formula is dvccorr::corr_backward.  Coordinates get no
        gradient (RAFTDVC.forward detaches them, raft_dvc.py:441).

Every op runs the HIP kernels of libdvccorr.so through ops.py (no CPU
fallback); the fake (meta) implementations only compute output shapes, so the
ops trace under torch.compile / FakeTensorMode and torch.library.opcheck.
`torch.utils.checkpoint(block, coords, use_reentrant=False)` (the reference's
checkpoint_corr path, raft_dvc.py:446-448) recomputes dvccorr::lookup_ad in the
backward pass.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from . import ops
from ._lib import layout

_F32 = torch.float32


def _n3(radius: int) -> int:
    return (2 * radius + 1) ** 3


@torch.library.custom_op("dvccorr::build", mutates_args=())
def build(packed_q: Tensor, packed_t: Tensor, C: int, H: int, W: int, D: int, num_levels: int,
          dtype: int) -> Tensor:
    return ops.build(packed_q, packed_t, C, H, W, D, num_levels, dtype, dtype)


@build.register_fake
def _(packed_q, packed_t, C, H, W, D, num_levels, dtype):
    # same metadata as ops.alloc_corr: a view past DVC_CORR_GUARD_BYTES of leading zeros
    lay = layout(H, W, D, num_levels, C)
    B, Nq, _ = packed_q.shape
    dt = ops._TORCH_DT[dtype]
    g = ops.GUARD_BYTES // torch.tensor([], dtype=dt).element_size()
    n = B * Nq * lay.row_stride
    return packed_q.new_empty((n + 2 * g,), dtype=dt)[g:g + n].view(B, Nq, lay.row_stride)


@torch.library.custom_op("dvccorr::lookup", mutates_args=())
def lookup(corr: Tensor, coords: Tensor, H: int, W: int, D: int, num_levels: int, radius: int, legacy: bool,
           dtype: int) -> Tensor:
    return ops.lookup(corr, coords, H, W, D, num_levels, radius, legacy, dtype)


@lookup.register_fake
def _(corr, coords, H, W, D, num_levels, radius, legacy, dtype):
    B, Nq, _ = corr.shape
    return corr.new_empty((B, num_levels * _n3(radius), Nq), dtype=_F32)


@torch.library.custom_op("dvccorr::lookup_fused", mutates_args=())
def lookup_fused(packed_q: Tensor, packed_t: Tensor, coords: Tensor, C: int, H: int, W: int, D: int,
                 num_levels: int, radius: int, legacy: bool, dtype: int) -> Tensor:
    return ops.lookup_fused(packed_q, packed_t, coords, C, H, W, D, num_levels, radius, legacy, dtype)


@lookup_fused.register_fake
def _(packed_q, packed_t, coords, C, H, W, D, num_levels, radius, legacy, dtype):
    B, Nq, _ = packed_q.shape
    return packed_q.new_empty((B, num_levels * _n3(radius), Nq), dtype=_F32)


@torch.library.custom_op("dvccorr::lookup_fused_proj", mutates_args=())
def lookup_fused_proj(packed_q: Tensor, packed_t: Tensor, coords: Tensor, packed_w: Tensor, bias: Tensor, C: int,
                      H: int, W: int, D: int, num_levels: int, radius: int, legacy: bool, dtype: int) -> Tensor:
    return ops.lookup_fused_proj(packed_q, packed_t, coords, packed_w, bias, C, H, W, D, num_levels, radius, legacy,
                                 dtype)


@lookup_fused_proj.register_fake
def _(packed_q, packed_t, coords, packed_w, bias, C, H, W, D, num_levels, radius, legacy, dtype):
    B, Nq, _ = packed_q.shape
    return packed_q.new_empty((B, 96, Nq), dtype=_F32)


@torch.library.custom_op("dvccorr::corr_backward", mutates_args=())
def corr_backward(packed_q: Tensor, packed_t: Tensor, coords: Tensor, grad_out: Tensor, C: int, H: int, W: int,
                  D: int, num_levels: int, radius: int, legacy: bool, dtype: int) -> tuple[Tensor, Tensor]:
    return ops.corr_backward(packed_q, packed_t, coords, grad_out, C, H, W, D, num_levels, radius, legacy, dtype)


@corr_backward.register_fake
def _(packed_q, packed_t, coords, grad_out, C, H, W, D, num_levels, radius, legacy, dtype):
    B, Nq, _ = packed_q.shape
    return (packed_q.new_empty((B, C, Nq), dtype=_F32), packed_q.new_empty((B, C, H, W, D), dtype=_F32))


@torch.library.custom_op("dvccorr::lookup_ad", mutates_args=())
def lookup_ad(fmap1: Tensor, fmap2: Tensor, corr: Optional[Tensor], packed_q: Tensor, packed_t: Tensor,
              coords: Tensor, C: int, H: int, W: int, D: int, num_levels: int, radius: int, legacy: bool,
              dtype: int) -> Tensor:
    if corr is not None:
        return ops.lookup(corr, coords, H, W, D, num_levels, radius, legacy, dtype)
    return ops.lookup_fused(packed_q, packed_t, coords, C, H, W, D, num_levels, radius, legacy, dtype)


@lookup_ad.register_fake
def _(fmap1, fmap2, corr, packed_q, packed_t, coords, C, H, W, D, num_levels, radius, legacy, dtype):
    B, Nq, _ = packed_q.shape
    return packed_q.new_empty((B, num_levels * _n3(radius), Nq), dtype=_F32)


def _lookup_ad_setup(ctx, inputs, output):
    fmap1, fmap2, _corr, q, t, coords, C, H, W, D, L, r, legacy, dtype = inputs
    ctx.save_for_backward(q, t, coords)
    ctx.geo = (C, H, W, D, L, r, legacy, dtype)
    ctx.fmap_meta = (tuple(fmap1.shape), fmap1.dtype, tuple(fmap2.shape), fmap2.dtype)


def _lookup_ad_backward(ctx, grad_out):
    q, t, coords = ctx.saved_tensors
    C, H, W, D, L, r, legacy, dtype = ctx.geo
    s1, dt1, s2, dt2 = ctx.fmap_meta
    d1, d2 = corr_backward(q, t, coords, grad_out.contiguous(), C, H, W, D, L, r, legacy, dtype)
    return (d1.view(s1).to(dt1), d2.view(s2).to(dt2)) + (None,) * 12


torch.library.register_autograd("dvccorr::lookup_ad", _lookup_ad_backward, setup_context=_lookup_ad_setup)


@torch.library.custom_op("dvccorr::lookup_convc1_ad", mutates_args=())
def lookup_convc1_ad(fmap1: Tensor, fmap2: Tensor, weight: Tensor, bias: Tensor, corr: Optional[Tensor],
                     packed_q: Optional[Tensor], packed_t: Optional[Tensor], coords: Tensor, packed_w: Tensor, C: int,
                     H: int, W: int,
                     D: int, num_levels: int, radius: int, legacy: bool, dtype: int, store_dtype: int) -> Tensor:
    """relu(convc1(lookup(coords))) (update.py:246 after corr.py:169-208) as a differentiable op.  The forward is the
    fused kernel (materialised: dvc_corr_lookup_proj on `corr`; on the fly: dvc_corr_lookup_fused_proj on the packed
    operands), so the L*(2r+1)^3-channel lookup tensor is neither written nor saved for the backward: the
    autograd context keeps the (B, 96, Nq) output and the coordinates only.  fmap1 / fmap2 / weight / bias are the
    gradient carriers (packed_w is weight's packed fp16 image)."""
    if corr is not None:
        return ops.lookup_proj(corr, coords, packed_w, bias, H, W, D, num_levels, radius, legacy, store_dtype)
    return ops.lookup_fused_proj(packed_q, packed_t, coords, packed_w, bias, C, H, W, D, num_levels, radius, legacy,
                                 dtype)


@lookup_convc1_ad.register_fake
def _(fmap1, fmap2, weight, bias, corr, packed_q, packed_t, coords, packed_w, C, H, W, D, num_levels, radius, legacy,
      dtype, store_dtype):
    B, _, Nq = coords.shape
    return coords.new_empty((B, 96, Nq), dtype=_F32)


def _lookup_convc1_setup(ctx, inputs, output):
    fmap1, fmap2, weight, bias, corr, q, t, coords, _pw, C, H, W, D, L, r, legacy, dtype, sdt = inputs
    ctx.save_for_backward(q, t, coords, weight, output, corr)
    ctx.geo = (C, H, W, D, L, r, legacy, dtype, sdt)
    ctx.meta = (tuple(fmap1.shape), fmap1.dtype, tuple(fmap2.shape), fmap2.dtype, tuple(bias.shape), bias.dtype)


def _lookup_convc1_backward(ctx, grad_out):
    """With y = relu(W x + b) per query (x = the lookup's L*(2r+1)^3 values): gy = dL/dy * [y > 0];
    dW = sum_q gy x^T, db = sum_q gy, dx = W^T gy, and dx goes through dvccorr::corr_backward to the fmaps.
    x is recomputed by the plain lookup kernel (one fp32 pass, freed after dW) instead of being saved by the
    forward: the Trainer's twelve iterations keep 12 x (B, 96, Nq) instead of 12 x (B, L*(2r+1)^3, Nq)."""
    q, t, coords, weight, out, corr = ctx.saved_tensors
    C, H, W, D, L, r, legacy, dtype, sdt = ctx.geo
    s1, dt1, s2, dt2, sb, dtb = ctx.meta
    gy = grad_out.contiguous() * (out > 0)
    x = (ops.lookup(corr, coords, H, W, D, L, r, legacy, sdt) if corr is not None else
         ops.lookup_fused(q, t, coords, C, H, W, D, L, r, legacy, dtype))         # (B, K, Nq) fp32
    w2 = weight.detach().reshape(weight.shape[0], -1).float()                         # (96, K)
    dw = torch.einsum("bon,bkn->ok", gy, x).reshape(weight.shape).to(weight.dtype)
    del x
    db = gy.sum(dim=(0, 2)).reshape(sb).to(dtb)
    d1 = d2 = None
    if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:   # (the block's fmaps require grad: q / t were kept)
        dx = torch.einsum("ok,bon->bkn", w2, gy).contiguous()
        d1, d2 = corr_backward(q, t, coords, dx, C, H, W, D, L, r, legacy, dtype)
        d1, d2 = d1.view(s1).to(dt1), d2.view(s2).to(dt2)
    return (d1, d2, dw, db) + (None,) * 14


torch.library.register_autograd("dvccorr::lookup_convc1_ad", _lookup_convc1_backward,
                                setup_context=_lookup_convc1_setup)

__all__ = ["build", "lookup", "lookup_fused", "lookup_fused_proj", "corr_backward", "lookup_ad", "lookup_convc1_ad"]
