"""Python face of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker.  The product package
(raft-dvc_amd/dvccorr) never imports it.

Wraps oracle/corr_oracle.c (a float64 restatement of the reference
zachtong/RAFT-DVC src/core/corr.py; see that file's header for line
citations) through ctypes.  All arrays are numpy; inputs follow the
reference's layouts:
    fmap1, fmap2 : (B, C, H, W, D) float32            (corr.py:116-123)
    coords       : (B, 3, H, W, D) float32, (h, w, d)  (corr.py:169-178)
    lookup out   : (B, L*(2r+1)**3, H, W, D)          (corr.py:207-208)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    """Compile the C oracle with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(
                os.path.join(_HERE, "corr_oracle.c")):
            build()
        L = ctypes.CDLL(_SO)
        i64p = ctypes.POINTER(ctypes.c_longlong)
        fp = ctypes.POINTER(ctypes.c_float)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        c_int = ctypes.c_int
        L.oracle_levels.argtypes = [c_int, c_int, c_int, c_int, ip]
        L.oracle_levels.restype = c_int
        L.oracle_pyr_elems.argtypes = [c_int, c_int, c_int, c_int]
        L.oracle_pyr_elems.restype = ctypes.c_longlong
        L.oracle_corr_rows.argtypes = [fp, fp, c_int, c_int, c_int, c_int, c_int, c_int, i64p,
                                       ctypes.c_longlong, dp]
        L.oracle_corr_rows.restype = c_int
        L.oracle_lookup_rows.argtypes = [dp, i64p, ctypes.c_longlong, fp, c_int, c_int, c_int, c_int,
                                         c_int, c_int, c_int, dp]
        L.oracle_lookup_rows.restype = c_int
        L.oracle_sample.argtypes = [fp, c_int, c_int, c_int, c_int, c_int, fp, c_int, c_int, c_int,
                                    c_int, dp]
        L.oracle_sample.restype = c_int
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def level_dims(H: int, W: int, D: int, L: int):
    """Per-level (H_l, W_l, D_l); raises RuntimeError where avg_pool3d would."""
    dims = (ctypes.c_int * (3 * max(L, 1)))()
    if lib().oracle_levels(H, W, D, L, dims) != 0:
        raise RuntimeError(f"pyramid of {L} levels cannot be built from ({H},{W},{D})")
    return [(dims[3 * l], dims[3 * l + 1], dims[3 * l + 2]) for l in range(L)]


def corr_rows(fmap1, fmap2, num_levels: int, rows) -> np.ndarray:
    """Pyramid rows [len(rows), sum_l N_l] (float64, natural layout per level)."""
    f1, f2 = _f32(fmap1), _f32(fmap2)
    B, C, H, W, D = f1.shape
    level_dims(H, W, D, num_levels)
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    P = lib().oracle_pyr_elems(H, W, D, num_levels)
    out = np.empty((len(rows), P), np.float64)
    rc = lib().oracle_corr_rows(_ptr(f1, ctypes.c_float), _ptr(f2, ctypes.c_float), B, C, H, W, D,
                                num_levels, _ptr(rows, ctypes.c_longlong), len(rows),
                                _ptr(out, ctypes.c_double))
    assert rc == 0
    return out


def split_levels(pyr_rows: np.ndarray, H: int, W: int, D: int, L: int):
    """Split concatenated rows into per-level arrays [nrows, H_l, W_l, D_l]."""
    out, off = [], 0
    for (h, w, d) in level_dims(H, W, D, L):
        n = h * w * d
        out.append(pyr_rows[:, off:off + n].reshape(-1, h, w, d))
        off += n
    return out


def lookup_rows(pyr_rows, rows, coords, num_levels: int, radius: int, legacy: bool) -> np.ndarray:
    """Lookup for the given rows -> [len(rows), L*(2r+1)**3] float64."""
    c = _f32(coords)
    B, three, H, W, D = c.shape
    assert three == 3
    pyr_rows = np.ascontiguousarray(pyr_rows, dtype=np.float64)
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    n3 = (2 * radius + 1) ** 3
    out = np.empty((len(rows), num_levels * n3), np.float64)
    rc = lib().oracle_lookup_rows(_ptr(pyr_rows, ctypes.c_double), _ptr(rows, ctypes.c_longlong),
                                  len(rows), _ptr(c, ctypes.c_float), B, H, W, D, num_levels, radius,
                                  int(bool(legacy)), _ptr(out, ctypes.c_double))
    assert rc == 0
    return out


def corr_lookup(fmap1, fmap2, coords, num_levels: int = 4, radius: int = 4, legacy: bool = False,
                rows=None) -> np.ndarray:
    """Build + lookup.  rows=None -> full (B, L*n3, H, W, D); else [len(rows), L*n3]."""
    B, C, H, W, D = np.shape(fmap1)
    N = H * W * D
    full = rows is None
    if full:
        rows = np.arange(B * N, dtype=np.int64)
    pyr = corr_rows(fmap1, fmap2, num_levels, rows)
    out = lookup_rows(pyr, rows, coords, num_levels, radius, legacy)
    if not full:
        return out
    return np.ascontiguousarray(out.reshape(B, N, -1).transpose(0, 2, 1)).reshape(B, -1, H, W, D)


def motion_convc1(lookup_out, weight, bias) -> np.ndarray:
    """MotionEncoder's first layer on a lookup output: relu(conv1x1(corr, W) + b), float64.

    Reference src/core/update.py:219-222 (Conv3d(L*(2r+1)**3, 96, kernel_size=1)) and :246
    (F.relu(self.convc1(corr))).  lookup_out (B, K, H, W, D), weight (96, K[, 1, 1, 1]),
    bias (96,) -> (B, 96, H, W, D)."""
    x = np.asarray(lookup_out, np.float64)
    B, K = x.shape[:2]
    w = np.asarray(weight, np.float64).reshape(-1, K)
    y = np.einsum("ok,bkn->bon", w, x.reshape(B, K, -1)) + np.asarray(bias, np.float64)[None, :, None]
    return np.maximum(y, 0.0).reshape(B, w.shape[0], *x.shape[2:])


def sample(vol, pts, legacy: bool = False) -> np.ndarray:
    """bilinear_sampler_3d: vol (B,C,H,W,D), pts (B,H',W',D',3) -> (B,C,H',W',D') float64."""
    v, p = _f32(vol), _f32(pts)
    B, C, H, W, D = v.shape
    _, Hq, Wq, Dq, three = p.shape
    assert three == 3 and p.shape[0] == B
    out = np.empty((B, C, Hq, Wq, Dq), np.float64)
    rc = lib().oracle_sample(_ptr(v, ctypes.c_float), B, C, H, W, D, _ptr(p, ctypes.c_float), Hq, Wq,
                             Dq, int(bool(legacy)), _ptr(out, ctypes.c_double))
    assert rc == 0
    return out


def coords_grid_3d(B: int, H: int, W: int, D: int) -> np.ndarray:
    """Identity grid (B, 3, H, W, D) float32, channel c = index along axis c (corr.py:91-97)."""
    g = np.stack(np.meshgrid(np.arange(H), np.arange(W), np.arange(D), indexing="ij"), 0).astype(np.float32)
    return np.ascontiguousarray(np.broadcast_to(g[None], (B, 3, H, W, D)))


def _axis_weights(n_in: int, n_out: int):
    """ATen CPU linear-upsample indices/weights, align_corners=True, in float32
    (area_pixel_compute_scale + compute_source_index_and_lambda), the arithmetic
    behind F.interpolate(mode='trilinear', align_corners=True) at corr.py:234-239."""
    ratio = np.float32(n_in - 1) / np.float32(n_out - 1) if n_out > 1 else np.float32(0.0)
    src = np.float32(ratio) * np.arange(n_out, dtype=np.float32)
    i0 = src.astype(np.int64)
    i1 = i0 + (i0 < n_in - 1)
    l1 = np.clip(src - i0.astype(np.float32), np.float32(0), np.float32(1)).astype(np.float32)
    return i0, i1, (np.float32(1) - l1).astype(np.float32), l1


def upflow_3d(flow, target_shape) -> np.ndarray:
    """upflow_3d (src/core/corr.py:211-253) restated in float32 numpy: trilinear,
    align_corners=True, nested h-outer (ATen's Interpolate<n>), then channel c < 3
    times float32(target/source) along axis c (corr.py:242-251)."""
    f = _f32(flow)
    B, C, h, w, d = f.shape
    H, W, D = target_shape
    yi0, yi1, yl0, yl1 = _axis_weights(h, H)
    xi0, xi1, xl0, xl1 = _axis_weights(w, W)
    zi0, zi1, zl0, zl1 = _axis_weights(d, D)

    def along_z(a):           # (B, C, h', w', d) -> (B, C, h', w', D)
        return a[..., zi0] * zl0 + a[..., zi1] * zl1

    def along_x(a0, a1):
        return a0 * xl0[:, None] + a1 * xl1[:, None]

    def plane(yi):             # (B, C, W, D) for source rows yi
        a = f[:, :, yi]        # (B, C, H, w, d)
        zx0 = along_z(a[:, :, :, xi0])
        zx1 = along_z(a[:, :, :, xi1])
        return along_x(zx0, zx1)

    out = plane(yi0) * yl0[:, None, None] + plane(yi1) * yl1[:, None, None]
    scale = [np.float32(H / h), np.float32(W / w), np.float32(D / d)]
    for c in range(min(C, 3)):
        out[:, c] *= scale[c]
    return out.astype(np.float32)


def flow_step(coords1, delta_flow, target_shape):
    """raft_dvc.py:482-485: coords1 + delta_flow, and upflow_3d(coords1 - coords0)."""
    c1 = _f32(coords1)
    if delta_flow is not None:
        c1 = (c1 + _f32(delta_flow)).astype(np.float32)
    B, _, h, w, d = c1.shape
    flow = (c1 - coords_grid_3d(B, h, w, d)).astype(np.float32)
    return c1, upflow_3d(flow, target_shape)


def rel_err(out, ref) -> float:
    """max|out - ref| / max|ref| -- the tolerance metric of SURVEY.md 8(c)."""
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    den = np.abs(ref).max() if ref.size else 0.0
    num = np.abs(out - ref).max() if ref.size else 0.0
    return float(num / den) if den > 0 else float(num)
