#!/usr/bin/env python3
"""Timeline of the convc1-fused tile lookup (diagnostics, round 6): thread 0 of every workgroup stamps
s_memrealtime (100 MHz) at checkpoints of EVERY level it walks (lookup_tile.h ABL & 16 instance,
k_lookup_tile<bf16, 4, .., PROJ=1>), 16 stamps per level:
  1 level start   2 window table published   3 plane 0 loaded + written   4 plane 0 visible
  5 plane 1 visible   6.. end of output row 0, 1, ...      (slot 3*16+15: workgroup end)

    python tools/trace_proj.py [--size 32]
Prints, per level position in the walk, per-phase duration quantiles (us) and the gap between the previous
level's last row and this level's first row (the per-level pipeline restart)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
os.environ.setdefault("DVCCORR_LIB", os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr_diag.so"))
import dvccorr  # noqa: E402
from dvccorr import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
coords = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
K = L * (2 * R + 1) ** 3
w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
bias = torch.zeros(96, device=dev)
with torch.no_grad():
    blk = dvccorr.CorrBlock(f1, f2, L, R, precision="bf16")
    for _ in range(3):
        blk.lookup_convc1(coords, w, bias)
    torch.cuda.synchronize()
    nwg = (S ** 3 + 63) // 64
    buf = torch.zeros(nwg * 64, dtype=torch.int64, device=dev)
    p = buf.data_ptr()
    _lib.set_tuning("lookup_trace_lo", int(p & 0xffffffff) - (1 << 32 if p & 0x80000000 else 0))
    _lib.set_tuning("lookup_trace_hi", int(p >> 32))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    blk.lookup_convc1(coords, w, bias)
    e1.record()
    torch.cuda.synchronize()
    _lib.set_tuning("lookup_trace_lo", 0)
    _lib.set_tuning("lookup_trace_hi", 0)
st = buf.view(nwg, 4, 16).cpu().numpy().astype(np.float64)
t0 = st[:, 0, 1][st[:, 0, 1] > 0].min()
rel = np.where(st > 0, (st - t0) / 100.0, np.nan)
q = lambda x: [round(float(v), 2) for v in np.nanpercentile(x, [0, 50, 90, 100])] if np.isfinite(x).any() else None
res = {"event_ms": round(e0.elapsed_time(e1), 4), "workgroups": int(nwg), "end_us": q(rel[:, 3, 15])}
names = {1: "start", 2: "table", 3: "plane0", 4: "plane0_vis", 5: "plane1_vis"}
for li in range(4):
    ph = {}
    prev = 1
    for k in range(2, 15):
        d = rel[:, li, k] - rel[:, li, prev]
        if np.isfinite(d).any():
            ph[f"{names.get(prev, f'row{prev - 6}')}->{names.get(k, f'row{k - 6}')}"] = q(d)
            prev = k
    if li > 0:
        last = np.nanmax(rel[:, li - 1, 6:15], axis=1)
        ph["prev_level_last_row->start"] = q(rel[:, li, 1] - last)
        ph["prev_level_last_row->row0"] = q(rel[:, li, 6] - last)
    ph["level_total(start->last_row)"] = q(np.nanmax(rel[:, li, 6:15], axis=1) - rel[:, li, 1])
    res[f"level_pos{li}"] = ph
print(json.dumps(res, indent=1))
