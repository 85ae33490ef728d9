"""ctypes binding of libdvccorr.so (the C ABI declared in include/dvccorr.h).

The shared library is built in-tree (raft-dvc_amd/csrc/Makefile, or
`python -c "import __graft_entry__ as g; g.build()"`) and loaded from this
directory.  There is no fallback: if the library is missing the import of the
product path fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DVCCORR_LIB (diagnostics): load another in-tree build of the same ABI, e.g. for A/B kernel timing
LIB_PATH = os.environ.get("DVCCORR_LIB") or os.path.join(_HERE, "libdvccorr.so")

DVC_OK, DVC_ERR_INVALID, DVC_ERR_UNSUPPORTED, DVC_ERR_LAUNCH, DVC_ERR_RUNTIME = range(5)
DVC_F32, DVC_BF16, DVC_F16 = 0, 1, 2
DVC_BRICKED = 0x100     # layout flag ORed into a dtype (include/dvccorr.h)
DVC_FIXED, DVC_LEGACY = 0, 1
MAX_LEVELS = 8

# Every symbol include/dvccorr.h declares (checked by tests/test_capi_cpu.py).
EXPORTED = (
    "dvc_layout_init", "dvc_pack_workspace_bytes", "dvc_pack_queries", "dvc_pack_targets", "dvc_pack_targets_gathered",
    "dvc_corr_build",
    "dvc_corr_pool", "dvc_corr_lookup", "dvc_lookup_fused_workspace_bytes", "dvc_corr_lookup_fused",
    "dvc_sample3d", "dvc_set_tuning", "dvc_last_error", "dvc_version", "dvc_abi_version",
    "dvc_corr_backward_workspace_bytes", "dvc_corr_backward_workspace_bytes_dtype", "dvc_corr_backward",
    "dvc_proj_packed_bytes", "dvc_proj_pack", "dvc_proj_pack_exact",
    "dvc_corr_lookup_proj", "dvc_lookup_fused_proj_workspace_bytes", "dvc_corr_lookup_fused_proj",
    "dvc_coords_grid", "dvc_upflow", "dvc_flow_step", "dvc_bricked_levels", "dvc_corr_backward_mfma", "dvc_corr_backward_gout64",
)
PROJ_COUT = 96          # DVC_PROJ_COUT (convc1 output channels, update.py:222)
PROJ_MAX_RADIUS = 4     # DVC_PROJ_MAX_RADIUS


class Layout(ctypes.Structure):
    """Mirror of dvc_layout."""
    _fields_ = [
        ("num_levels", ctypes.c_int32),
        ("channels", ctypes.c_int32),
        ("c_pad", ctypes.c_int32),
        ("H", ctypes.c_int32 * MAX_LEVELS),
        ("W", ctypes.c_int32 * MAX_LEVELS),
        ("D", ctypes.c_int32 * MAX_LEVELS),
        ("Dp", ctypes.c_int32 * MAX_LEVELS),
        ("zero_level", ctypes.c_int32 * MAX_LEVELS),
        ("offset", ctypes.c_int64 * MAX_LEVELS),
        ("level_elems", ctypes.c_int64 * MAX_LEVELS),
        ("row_elems", ctypes.c_int64),
        ("row_stride", ctypes.c_int64),
    ]

    def levels(self):
        return [(self.H[l], self.W[l], self.D[l]) for l in range(self.num_levels)]


class DvcError(RuntimeError):
    """A HIP launch/runtime failure reported by libdvccorr."""


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C raft-dvc_amd/csrc` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    i32, i64, vp, sz = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t
    sig = {
        "dvc_layout_init": (i32, [i32, i32, i32, i32, i32, ctypes.POINTER(Layout)]),
        "dvc_bricked_levels": (i32, [ctypes.POINTER(Layout)]),
        "dvc_pack_workspace_bytes": (sz, [i32, i32, i32, i32, i32, i32]),
        "dvc_pack_queries": (i32, [vp, vp, i32, i32, i64, i32, vp]),
        "dvc_pack_targets": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_pack_targets_gathered": (i32, [vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_corr_build": (i32, [vp, vp, vp, i32, i64, i32, i32, i32, i32, i32, i32, i32, i64, i64, vp]),
        "dvc_corr_pool": (i32, [vp, i32, i64, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_corr_lookup": (i32, [vp, vp, vp, i32, i64, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_lookup_fused_workspace_bytes": (sz, [i32, i64, i32, i32]),
        "dvc_corr_lookup_fused": (i32, [vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_sample3d": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i64, i32, vp]),
        "dvc_corr_backward_workspace_bytes": (sz, [i32, i64, i32, i32, i32, i32, i32, i32]),
        "dvc_corr_backward_workspace_bytes_dtype": (sz, [i32, i64, i32, i32, i32, i32, i32, i32, i32]),
        "dvc_corr_backward": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, i32, i32, i32, i32,
                                    vp]),
        "dvc_corr_backward_mfma": (i32, [i32, i64, i32, i32, i32, i32, i32, i32, i32, i32]),
        "dvc_corr_backward_gout64": (i32, [i64, i32]),
        "dvc_proj_packed_bytes": (sz, [i32, i32]),
        "dvc_proj_pack": (i32, [vp, vp, i32, i32, i32, i32, vp]),
        "dvc_proj_pack_exact": (i32, [vp, vp, i32, i32, i32, i32, vp]),
        "dvc_corr_lookup_proj": (i32, [vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_lookup_fused_proj_workspace_bytes": (sz, [i32, i64]),
        "dvc_corr_lookup_fused_proj": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, i32, i32, i32,
                                             i32, vp]),
        "dvc_coords_grid": (i32, [vp, i32, i32, i32, i32, vp]),
        "dvc_upflow": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_flow_step": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
        "dvc_set_tuning": (i32, [ctypes.c_char_p, i32]),
        "dvc_last_error": (ctypes.c_char_p, []),
        "dvc_version": (ctypes.c_char_p, []),
        "dvc_abi_version": (i32, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    """Turn a dvc_status into the exception the reference would raise."""
    if rc == DVC_OK:
        return
    msg = lib().dvc_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if rc == DVC_ERR_INVALID:
        raise ValueError(msg)
    if rc == DVC_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise DvcError(msg)


def set_tuning(key: str, value: int) -> None:
    check(lib().dvc_set_tuning(key.encode(), int(value)), "set_tuning")


def layout(H: int, W: int, D: int, num_levels: int, C: int = 1) -> Layout:
    """Pyramid geometry.  Raises RuntimeError where the reference's avg_pool3d would."""
    lay = Layout()
    rc = lib().dvc_layout_init(H, W, D, num_levels, C, ctypes.byref(lay))
    if rc != DVC_OK:
        raise RuntimeError(lib().dvc_last_error().decode(errors="replace"))
    return lay


def bricked_levels(lay: Layout) -> int:
    """Bit mask of the levels a DVC_BRICKED pyramid stores in (1, 8, 8) bricks."""
    return int(lib().dvc_bricked_levels(ctypes.byref(lay)))
