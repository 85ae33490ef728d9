#!/usr/bin/env python3
"""Timeline of the default tile lookup (diagnostics): thread 0 of every workgroup stamps s_memrealtime
(100 MHz) at checkpoints of the first level it processes (lookup_tile.h, ABL & 8 instances):
  0 kernel start   1 level start (LDS cleared, coords loaded)   2 window table published
  3 chunk setup done, plane 0 loaded + written   4 plane 0 visible   5 plane 1 visible
  6.. end of output row 0, 1, ...   15 workgroup end

    python tools/trace_lookup.py [--shard-of 8] [--size 32]
Prints per-checkpoint quantiles (us) relative to the earliest workgroup start, and per-phase durations."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
# the diagnostics knobs (ablations, traces, store policies) live in libdvccorr_diag.so (make -C raft-dvc_amd/csrc diag)
os.environ.setdefault("DVCCORR_LIB", os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr_diag.so"))
from dvccorr import _lib, ops  # noqa: E402
from dvccorr.sharded import slab_bounds  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shard-of", type=int, default=1)
ap.add_argument("--size", type=int, default=32)
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
h0, h1 = slab_bounds(S, a.shard_of, 0)
base = torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
coords = (base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2))[:, :, h0:h1].contiguous().to(dev)
dt = ops.dtype_code("bf16")
lay = ops.layout(S, S, S, L, C)
brick = ops.DVC_BRICKED if ops.bricked_levels(lay) else 0
q = ops.pack_queries(f1[:, :, h0:h1].reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt | brick)
corr = ops.build(q, t, C, S, S, S, L, dt, dt)
cf = coords.reshape(1, 3, -1)
for _ in range(3):
    ops.lookup(corr, cf, S, S, S, L, R, False, dt | brick)
nwg = 8192
buf = torch.zeros(nwg * 16, dtype=torch.int64, device=dev)
p = buf.data_ptr()
_lib.set_tuning("lookup_trace_lo", int(p & 0xffffffff) - (1 << 32 if p & 0x80000000 else 0))
_lib.set_tuning("lookup_trace_hi", int(p >> 32))
ops.lookup(corr, cf, S, S, S, L, R, False, dt | brick)
torch.cuda.synchronize()
_lib.set_tuning("lookup_trace_lo", 0)
_lib.set_tuning("lookup_trace_hi", 0)
st = buf.view(nwg, 16).cpu().numpy().astype(np.float64)
used = st[:, 0] > 0
st = st[used]
t0 = st[:, 0].min()
rel = np.where(st > 0, (st - t0) / 100.0, np.nan)   # us (100 MHz)
res = {"shard_of": a.shard_of, "workgroups": int(used.sum()), "kernel_us": float(np.nanmax(rel[:, 15]))}
names = ["start", "level", "table", "plane0", "plane0_vis", "plane1_vis"] + [f"row{i}" for i in range(9)] + ["end"]
q = lambda x: [round(float(v), 2) for v in np.nanpercentile(x, [0, 50, 90, 100])] if np.isfinite(x).any() else None
res["at_us_q0_50_90_100"] = {names[k]: q(rel[:, k]) for k in range(16)}
ph = {}
prev = 0
for k in range(1, 15):
    d = rel[:, k] - rel[:, prev]
    if np.isfinite(d).any():
        ph[f"{names[prev]}->{names[k]}"] = q(d)
        prev = k
ph["last->end"] = q(rel[:, 15] - np.nanmax(rel[:, 1:15], axis=1))
res["phase_us_q0_50_90_100"] = ph
print(json.dumps(res, indent=1))
