"""dvccorr -- MI355X-native correlation hot path for RAFT-DVC.

Drop-in replacements for the reference's src/core/corr.py / corr_otf.py
objects (see corr_block.py), backed by hand-written gfx950 HIP kernels in
libdvccorr.so behind the C ABI of include/dvccorr.h, plus the query-voxel
sharded block for multi-GPU runs (sharded.py).
"""
from __future__ import annotations

from ._lib import LIB_PATH, DvcError, layout
from .corr_block import (CorrBlock, CorrBlockFused, CorrBlockOnTheFly, bilinear_sampler_3d, coords_grid_3d,
                         flow_step, make_corr_block, resolve_precision, upflow_3d)

__version__ = "0.1.0"

__all__ = ["CorrBlock", "CorrBlockFused", "CorrBlockOnTheFly", "bilinear_sampler_3d", "coords_grid_3d",
           "upflow_3d", "flow_step", "make_corr_block", "resolve_precision", "layout", "DvcError", "LIB_PATH"]
