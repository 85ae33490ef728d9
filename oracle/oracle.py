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


def rel_err(out, ref) -> float:
    """max|out - ref| / max|ref| -- the tolerance metric of SURVEY.md 8(c)."""
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    den = np.abs(ref).max() if ref.size else 0.0
    num = np.abs(out - ref).max() if ref.size else 0.0
    return float(num / den) if den > 0 else float(num)
