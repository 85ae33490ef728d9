"""Tensor-level wrappers over the C ABI.

PyTorch supplies device memory and the current HIP stream; every call goes
straight to libdvccorr.so (no CPU fallback).  Shapes follow include/dvccorr.h:

    pack_queries(fmap1_slab (B, C, Nq) f32)            -> (B, Nq, Cp)          dtype
    pack_targets(fmap2 (B, C, H, W, D) f32, L)         -> (B, row_stride, Cp)  dtype
    build(q, t, ...)                                   -> (B, Nq, row_stride)  store dtype
    pool(corr, ..., src_level)                         in place
    lookup(corr, coords (B, 3, Nq) f32, ...)           -> (B, L*(2r+1)^3, Nq)  f32
    lookup_fused(q, t, coords, ...)                    -> (B, L*(2r+1)^3, Nq)  f32
    sample3d(vol (B, C, Hv, Wv, Dv), pts (B, Nq, 3))   -> (B, C, Nq)           f32
    proj_pack(convc1 weight (96, L*(2r+1)^3) f32, ...) -> packed fp16 weights
    lookup_proj(corr, coords, packed_w, bias, ...)     -> (B, 96, Nq)          f32
    coords_grid(B, H, W, D, device)                    -> (B, 3, H, W, D)      f32
    upflow(flow (B, C, h, w, d), (H, W, D))            -> (B, C, H, W, D)      f32
    flow_step(coords1, delta (B, 3, h, w, d), (H,W,D)) -> coords1 + delta, upflow(coords1 + delta - coords0)
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import DVC_BF16, DVC_BRICKED, DVC_F16, DVC_F32, DVC_FIXED, DVC_LEGACY, bricked_levels, check, layout, lib


class _DtypeMap(dict):
    """dtype code -> torch dtype; a DVC_BRICKED layout flag ORed into the code is ignored."""

    def __getitem__(self, code):
        return super().__getitem__(int(code) & ~DVC_BRICKED)


_TORCH_DT = _DtypeMap({DVC_F32: torch.float32, DVC_BF16: torch.bfloat16, DVC_F16: torch.float16})


def dtype_code(precision: str) -> int:
    if precision in ("fp32", "float32", "f32"):
        return DVC_F32
    if precision in ("bf16", "bfloat16"):
        return DVC_BF16
    if precision in ("fp16", "float16", "f16", "half"):
        return DVC_F16
    raise ValueError(f"precision must be 'fp32', 'bf16' or 'fp16', got {precision!r}")


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def _stream(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)



def _on_device(fn):
    """Run an op with its tensors' device current (torch.cuda.device), so the C ABI's launches, workspaces and
    the backward's side stream land on the GPU that owns the data even when the calling thread's current device
    is another one (a block on cuda:1 driven from a thread whose current device is 0)."""
    import functools

    @functools.wraps(fn)
    def run(*args, **kwargs):
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, torch.Tensor) and a.is_cuda:
                with torch.cuda.device(a.device):
                    return fn(*args, **kwargs)
        return fn(*args, **kwargs)

    return run


def _need_cuda(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("dvccorr runs on the MI355X only: got a CPU tensor (no CPU fallback)")


def _mark(t: torch.Tensor, dtype: int) -> torch.Tensor:
    """Record the DVC_BRICKED layout flag next to a packed-target / pyramid buffer (the C ABI cannot tell)."""
    t._dvc_bricked = bool(int(dtype) & DVC_BRICKED)
    return t


def _expect_layout(t: torch.Tensor, dtype: int, what: str) -> None:
    """A buffer packed bricked must be read with DVC_BRICKED, and only by the entry points that take it."""
    rec = getattr(t, "_dvc_bricked", None)
    if rec is not None and rec != bool(int(dtype) & DVC_BRICKED):
        raise ValueError(f"{what}: the buffer was packed {'bricked' if rec else 'linear'} but is passed as "
                         f"{'bricked' if int(dtype) & DVC_BRICKED else 'linear'} (include/dvccorr.h, DVC_BRICKED)")


def _f32c(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.float32).contiguous()


@_on_device
def pack_queries(fmap1_slab: torch.Tensor, dtype: int) -> torch.Tensor:
    _need_cuda(fmap1_slab)
    f = _f32c(fmap1_slab)
    B, C, Nq = f.shape
    Cp = 32 if C <= 32 else 64 if C <= 64 else (C + 127) // 128 * 128   # dvc_layout_init's c_pad
    out = torch.empty((B, Nq, Cp), dtype=_TORCH_DT[dtype], device=f.device)
    check(lib().dvc_pack_queries(_ptr(f), _ptr(out), B, C, Nq, dtype, _stream(f)), "pack_queries")
    return out


@_on_device
def pack_targets(fmap2: torch.Tensor, num_levels: int, dtype: int, out: torch.Tensor = None) -> torch.Tensor:
    """fmap2 -> packed targets of every level; dtype | DVC_BRICKED stores the bricked levels in brick order
    (the materialised build then writes a bricked pyramid, which only the tile lookups read)."""
    _need_cuda(fmap2)
    f = _f32c(fmap2)
    B, C, H, W, D = f.shape
    lay = layout(H, W, D, num_levels, C)
    if out is None:
        out = torch.empty((B, lay.row_stride, lay.c_pad), dtype=_TORCH_DT[dtype], device=f.device)
    nws = lib().dvc_pack_workspace_bytes(B, C, H, W, D, num_levels)
    ws = torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=f.device)
    check(lib().dvc_pack_targets(_ptr(f), _ptr(out), _ptr(ws), B, C, H, W, D, num_levels, dtype, _stream(f)),
          "pack_targets")
    return _mark(out, dtype)


@_on_device
def pack_targets_gathered(gathered: torch.Tensor, H: int, num_levels: int, dtype: int) -> torch.Tensor:
    """pack_targets of the fmap2 an H-slab all-gather delivers, read from its receive buffer
    gathered (world, B, C, ceil(H / world), W, D) without assembling fmap2 (dvc_pack_targets_gathered;
    sharded.all_gather_slab's buffer, slab r = slab_bounds(H, world, r), zero-padded)."""
    _need_cuda(gathered)
    if gathered.dtype != torch.float32 or not gathered.is_contiguous() or gathered.dim() != 6:
        raise ValueError("pack_targets_gathered: expected a contiguous float32 (world, B, C, maxh, W, D) buffer")
    world, B, C, maxh, W, D = gathered.shape
    if maxh != -(-H // world):
        raise ValueError(f"pack_targets_gathered: slab height {maxh} != ceil({H} / {world})")
    lay = layout(H, W, D, num_levels, C)
    out = torch.empty((B, lay.row_stride, lay.c_pad), dtype=_TORCH_DT[dtype], device=gathered.device)
    check(lib().dvc_pack_targets_gathered(_ptr(gathered), world, _ptr(out), B, C, H, W, D, num_levels, dtype,
                                          _stream(gathered)), "pack_targets_gathered")
    return _mark(out, dtype)


GUARD_BYTES = 256   # DVC_CORR_GUARD_BYTES


def alloc_corr(B: int, Nq: int, row_stride: int, store_dtype: int, device, zero: bool = False) -> torch.Tensor:
    """(B, Nq, row_stride) corr buffer with DVC_CORR_GUARD_BYTES of guard space on both sides (dvc_corr_build
    zeroes the guards; zero=True zeroes the whole buffer, for the pooled build whose build call covers only
    level 0's columns)."""
    dt = _TORCH_DT[store_dtype]
    g = GUARD_BYTES // torch.tensor([], dtype=dt).element_size()
    n = B * Nq * row_stride
    buf = (torch.zeros if zero else torch.empty)((n + 2 * g,), dtype=dt, device=device)
    return buf[g:g + n].view(B, Nq, row_stride)


@_on_device
def build(packed_q: torch.Tensor, packed_t: torch.Tensor, C: int, H: int, W: int, D: int, num_levels: int,
          in_dtype: int, store_dtype: int, col_begin: int = 0, col_end=None, out: torch.Tensor = None) -> torch.Tensor:
    _need_cuda(packed_q, packed_t)
    B, Nq, _ = packed_q.shape
    lay = layout(H, W, D, num_levels, C)
    col_end = lay.row_stride if col_end is None else col_end
    if out is None:
        out = alloc_corr(B, Nq, lay.row_stride, store_dtype, packed_q.device)
    check(lib().dvc_corr_build(_ptr(packed_q), _ptr(packed_t), _ptr(out), B, Nq, C, H, W, D, num_levels, in_dtype,
                               store_dtype, col_begin, col_end, _stream(packed_q)), "corr_build")
    # the build is layout-blind: bricked packed targets give a bricked pyramid
    out._dvc_bricked = getattr(packed_t, "_dvc_bricked", False)
    return out


@_on_device
def pool(corr: torch.Tensor, H: int, W: int, D: int, num_levels: int, src_level: int, store_dtype: int) -> None:
    _need_cuda(corr)
    _expect_layout(corr, store_dtype, "corr_pool")
    B, Nq, _ = corr.shape
    check(lib().dvc_corr_pool(_ptr(corr), B, Nq, H, W, D, num_levels, src_level, store_dtype, _stream(corr)),
          "corr_pool")


@_on_device
def lookup(corr: torch.Tensor, coords: torch.Tensor, H: int, W: int, D: int, num_levels: int, radius: int,
           legacy: bool, store_dtype: int, out: torch.Tensor = None) -> torch.Tensor:
    _need_cuda(corr, coords)
    _expect_layout(corr, store_dtype, "corr_lookup")
    B, Nq, _ = corr.shape
    c = _f32c(coords)
    n3 = (2 * radius + 1) ** 3
    if out is None:
        out = torch.empty((B, num_levels * n3, Nq), dtype=torch.float32, device=corr.device)
    check(lib().dvc_corr_lookup(_ptr(corr), _ptr(c), _ptr(out), B, Nq, H, W, D, num_levels, radius,
                                DVC_LEGACY if legacy else DVC_FIXED, store_dtype, _stream(corr)), "corr_lookup")
    return out


@_on_device
def proj_pack(weight: torch.Tensor, num_levels: int, radius: int, legacy: bool, exact: bool = False) -> torch.Tensor:
    """convc1.weight (96, L*(2r+1)^3[, 1, 1, 1]) -> the fused kernel's packed fp16 operand (dvc_proj_pack), or for
    fp32 pyramids (exact=True) its bf16 hi + lo blocks (dvc_proj_pack_exact, twice the bytes)."""
    _need_cuda(weight)
    w = _f32c(weight.detach().reshape(weight.shape[0], -1))
    nbytes = lib().dvc_proj_packed_bytes(num_levels, radius)
    if nbytes == 0:
        raise NotImplementedError(f"proj_pack: L={num_levels} r={radius} not supported (radius 1..4)")
    if w.shape[1] != num_levels * (2 * radius + 1) ** 3:
        raise ValueError(f"convc1 weight has {w.shape[1]} input channels; the lookup has "
                         f"{num_levels * (2 * radius + 1) ** 3}")
    out = torch.empty(((2 if exact else 1) * nbytes // 2,), dtype=torch.float16, device=w.device)
    fn = lib().dvc_proj_pack_exact if exact else lib().dvc_proj_pack
    check(fn(_ptr(w), _ptr(out), w.shape[0], num_levels, radius, DVC_LEGACY if legacy else DVC_FIXED, _stream(w)),
          "proj_pack")
    return out


_PACK_CACHE: dict = {}


def proj_pack_cached(weight: torch.Tensor, num_levels: int, radius: int, legacy: bool,
                     exact: bool = False) -> torch.Tensor:
    """proj_pack, re-packed only when the weight changes: the packing is once per optimiser step, not once
    per lookup.  Entries belong to the weight tensor OBJECT (a weak reference, checked on every hit, and a
    finalizer that drops the entry), plus its in-place version counter and shape, so a new weight that
    lands on a freed weight's address never reuses the old packing."""
    import weakref
    key = (id(weight), num_levels, radius, bool(legacy), bool(exact))
    hit = _PACK_CACHE.get(key)
    state = (weight._version, tuple(weight.shape), weight.device, weight.data_ptr())
    if hit is not None and hit[0]() is weight and hit[1] == state:
        return hit[2]
    packed = proj_pack(weight, num_levels, radius, legacy, exact)
    if hit is None or hit[0]() is not weight:
        weakref.finalize(weight, _PACK_CACHE.pop, key, None)
    _PACK_CACHE[key] = (weakref.ref(weight), state, packed)
    return packed


@_on_device
def lookup_proj(corr: torch.Tensor, coords: torch.Tensor, packed_w: torch.Tensor, bias: torch.Tensor, H: int, W: int,
                D: int, num_levels: int, radius: int, legacy: bool, store_dtype: int,
                out: torch.Tensor = None) -> torch.Tensor:
    """relu(convc1(lookup(coords))) -> (B, 96, Nq) f32, the lookup never written (dvc_corr_lookup_proj)."""
    _need_cuda(corr, coords, packed_w, bias)
    _expect_layout(corr, store_dtype, "corr_lookup_proj")
    B, Nq, _ = corr.shape
    c = _f32c(coords)
    b = _f32c(bias)
    if b.numel() != _lib.PROJ_COUT:
        raise ValueError(f"convc1 bias must have {_lib.PROJ_COUT} entries; got {b.numel()}")
    need = lib().dvc_proj_packed_bytes(num_levels, radius) * (2 if (int(store_dtype) & ~DVC_BRICKED) == DVC_F32 else 1)
    have = packed_w.numel() * packed_w.element_size()
    if have < need:
        raise ValueError(f"lookup_proj: packed_w holds {have} bytes; this store dtype's consumer reads {need} "
                         f"(fp32 pyramids take proj_pack(..., exact=True); include/dvccorr.h, ABI 3)")
    if out is None:
        out = torch.empty((B, _lib.PROJ_COUT, Nq), dtype=torch.float32, device=corr.device)
    check(lib().dvc_corr_lookup_proj(_ptr(corr), _ptr(c), _ptr(packed_w), _ptr(b), _ptr(out), B, Nq, H, W, D,
                                     num_levels, radius, DVC_LEGACY if legacy else DVC_FIXED, store_dtype,
                                     _stream(corr)), "corr_lookup_proj")
    return out


@_on_device
def lookup_fused_proj(packed_q: torch.Tensor, packed_t: torch.Tensor, coords: torch.Tensor, packed_w: torch.Tensor,
                      bias: torch.Tensor, C: int, H: int, W: int, D: int, num_levels: int, radius: int, legacy: bool,
                      dtype: int, out: torch.Tensor = None, workspace: torch.Tensor = None) -> torch.Tensor:
    """relu(convc1(lookup_fused(coords))) -> (B, 96, Nq) f32 on the on-the-fly path, the lookup never written
    (dvc_corr_lookup_fused_proj: queries grouped by window origin, convc1 on MFMA)."""
    _need_cuda(packed_q, packed_t, coords, packed_w, bias)
    _expect_layout(packed_t, dtype, "corr_lookup_fused_proj")
    B, Nq, _ = packed_q.shape
    c = _f32c(coords)
    b = _f32c(bias)
    if b.numel() != _lib.PROJ_COUT:
        raise ValueError(f"convc1 bias must have {_lib.PROJ_COUT} entries; got {b.numel()}")
    if out is None:
        out = torch.empty((B, _lib.PROJ_COUT, Nq), dtype=torch.float32, device=packed_q.device)
    nws = lib().dvc_lookup_fused_proj_workspace_bytes(B, Nq)
    if workspace is None or workspace.numel() * workspace.element_size() < nws:
        workspace = torch.empty((max(nws, 256),), dtype=torch.uint8, device=packed_q.device)
    check(lib().dvc_corr_lookup_fused_proj(_ptr(packed_q), _ptr(packed_t), _ptr(c), _ptr(packed_w), _ptr(b), _ptr(out),
                                           _ptr(workspace), B, Nq, C, H, W, D, num_levels, radius,
                                           DVC_LEGACY if legacy else DVC_FIXED, dtype, _stream(packed_q)),
          "corr_lookup_fused_proj")
    return out


@_on_device
def lookup_fused(packed_q: torch.Tensor, packed_t: torch.Tensor, coords: torch.Tensor, C: int, H: int, W: int,
                 D: int, num_levels: int, radius: int, legacy: bool, dtype: int, out: torch.Tensor = None,
                 workspace: torch.Tensor = None) -> torch.Tensor:
    _need_cuda(packed_q, packed_t, coords)
    _expect_layout(packed_t, dtype, "corr_lookup_fused")
    B, Nq, _ = packed_q.shape
    c = _f32c(coords)
    n3 = (2 * radius + 1) ** 3
    if out is None:
        out = torch.empty((B, num_levels * n3, Nq), dtype=torch.float32, device=packed_q.device)
    nws = lib().dvc_lookup_fused_workspace_bytes(B, Nq, num_levels, radius)
    if workspace is None or workspace.numel() * workspace.element_size() < nws:
        workspace = torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=packed_q.device)
    check(lib().dvc_corr_lookup_fused(_ptr(packed_q), _ptr(packed_t), _ptr(c), _ptr(out), _ptr(workspace), B, Nq, C,
                                      H, W, D, num_levels, radius, DVC_LEGACY if legacy else DVC_FIXED, dtype,
                                      _stream(packed_q)), "corr_lookup_fused")
    return out


def fused_workspace(B: int, Nq: int, num_levels: int, radius: int, device) -> torch.Tensor:
    nws = lib().dvc_lookup_fused_workspace_bytes(B, Nq, num_levels, radius)
    return torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=device)


@_on_device
def corr_backward(packed_q: torch.Tensor, packed_t: torch.Tensor, coords: torch.Tensor, grad_out: torch.Tensor,
                  C: int, H: int, W: int, D: int, num_levels: int, radius: int, legacy: bool, dtype: int):
    """d loss / d fmap1 (B, C, Nq) and d loss / d fmap2 (B, C, H, W, D), both float32, from the gradient of
    a lookup output (B, L*(2r+1)^3, Nq) (dvc_corr_backward)."""
    _need_cuda(packed_q, packed_t, coords, grad_out)
    _expect_layout(packed_t, dtype, "corr_backward")
    B, Nq, _ = packed_q.shape
    c = _f32c(coords)
    g = _f32c(grad_out)
    dev = packed_q.device
    d1 = torch.empty((B, C, Nq), dtype=torch.float32, device=dev)
    d2 = torch.empty((B, C, H, W, D), dtype=torch.float32, device=dev)
    nws = lib().dvc_corr_backward_workspace_bytes_dtype(B, Nq, C, H, W, D, num_levels, radius, dtype)
    ws = torch.empty((max(nws, 256),), dtype=torch.uint8, device=dev)
    check(lib().dvc_corr_backward(_ptr(packed_q), _ptr(packed_t), _ptr(c), _ptr(g), _ptr(d1), _ptr(d2), _ptr(ws), B,
                                  Nq, C, H, W, D, num_levels, radius, DVC_LEGACY if legacy else DVC_FIXED, dtype,
                                  _stream(packed_q)), "corr_backward")
    return d1, d2


@_on_device
def sample3d(vol: torch.Tensor, pts: torch.Tensor, legacy: bool) -> torch.Tensor:
    _need_cuda(vol, pts)
    v = _f32c(vol)
    p = _f32c(pts)
    B, C, Hv, Wv, Dv = v.shape
    Nq = p.numel() // (3 * B)
    out = torch.empty((B, C, Nq), dtype=torch.float32, device=v.device)
    check(lib().dvc_sample3d(_ptr(v), _ptr(p), _ptr(out), B, C, Hv, Wv, Dv, Nq,
                             DVC_LEGACY if legacy else DVC_FIXED, _stream(v)), "sample3d")
    return out


def coords_grid(B: int, H: int, W: int, D: int, device) -> torch.Tensor:
    out = torch.empty((B, 3, H, W, D), dtype=torch.float32, device=device)
    _need_cuda(out)
    with torch.cuda.device(out.device):
        check(lib().dvc_coords_grid(_ptr(out), B, H, W, D, _stream(out)), "coords_grid")
    return out


@_on_device
def upflow(flow: torch.Tensor, target_shape) -> torch.Tensor:
    _need_cuda(flow)
    f = _f32c(flow)
    if f.dim() != 5:
        raise ValueError(f"upflow_3d expects (B, C, H, W, D), got {tuple(f.shape)}")
    B, C, h, w, d = f.shape
    H, W, D = (int(v) for v in target_shape)
    out = torch.empty((B, C, H, W, D), dtype=torch.float32, device=f.device)
    check(lib().dvc_upflow(_ptr(f), _ptr(out), B, C, h, w, d, H, W, D, _stream(f)), "upflow")
    return out


@_on_device
def flow_step(coords1: torch.Tensor, delta_flow, target_shape):
    """(coords1 + delta_flow, upflow_3d(coords1 + delta_flow - coords0, target_shape)) in one pass."""
    _need_cuda(coords1)
    c = _f32c(coords1)
    if c.dim() != 5 or c.shape[1] != 3:
        raise ValueError(f"coords1 must be (B, 3, H, W, D), got {tuple(c.shape)}")
    B, _, h, w, d = c.shape
    H, W, D = (int(v) for v in target_shape)
    dl = None
    if delta_flow is not None:
        _need_cuda(delta_flow)
        dl = _f32c(delta_flow)
        if dl.shape != c.shape:
            raise ValueError(f"delta_flow {tuple(dl.shape)} does not match coords1 {tuple(c.shape)}")
    new = torch.empty_like(c)
    up = torch.empty((B, 3, H, W, D), dtype=torch.float32, device=c.device)
    check(lib().dvc_flow_step(_ptr(c), None if dl is None else _ptr(dl), _ptr(new), _ptr(up), B, h, w, d, H, W, D,
                              _stream(c)), "flow_step")
    return new, up


__all__ = ["pack_queries", "pack_targets", "pack_targets_gathered", "build", "pool", "lookup", "lookup_fused", "lookup_fused_proj", "corr_backward", "sample3d",
           "proj_pack", "proj_pack_cached", "lookup_proj",
           "coords_grid", "upflow", "flow_step",
           "fused_workspace", "dtype_code", "layout", "bricked_levels", "DVC_BRICKED", "_lib"]
