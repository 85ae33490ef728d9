#!/usr/bin/env python3
"""Time the bf16 build kernel alone (HIP events) under tuning knobs / ablations.

    python tools/build_ab.py [--size 32] [--reps 10] [--knobs "build_ablate=1;build_ablate=2"]"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
import dvccorr  # noqa: E402
from dvccorr import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--knobs", default="", help="';'-separated settings, each a ','-list of key=value")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, L, C = a.size, a.levels, 128
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
dt = ops.dtype_code("bf16")
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
lay = dvccorr.layout(S, S, S, L, C)
out = ops.alloc_corr(1, S ** 3, lay.row_stride, dt, dev)
nbytes = S ** 3 * sum(h * w * d for h, w, d in lay.levels()) * 2
res = {}
for setting in [""] + [x for x in a.knobs.split(";") if x]:
    kv = [x.split("=") for x in setting.split(",") if x]
    for k, v in kv:
        _lib.set_tuning(k, int(v))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for r in range(a.reps + 2):
        e0.record()
        ops.build(q, t, C, S, S, S, L, dt, dt, out=out)
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    for k, v in kv:
        _lib.set_tuning(k, 0)
    m = statistics.median(ts)
    res[setting or "default"] = {"median_ms": m, "min_ms": min(ts), "GB/s": nbytes / (m * 1e-3) / 1e9}
print(json.dumps(res))
