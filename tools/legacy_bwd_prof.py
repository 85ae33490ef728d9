#!/usr/bin/env python3
"""Workload for a rocprofv3 kernel trace of the backward on a legacy non-cubic level set (tools/bench_legacy.py's
shape): `reps` dvc_corr_backward calls, legacy and fixed convention."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
import dvccorr  # noqa: E402
from dvccorr import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="32,32,16")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--legacy", type=int, default=1)
a = ap.parse_args()
H, W, D = (int(x) for x in a.shape.split(","))
dev = torch.device("cuda:0")
C, L, R = 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(11)
f1 = torch.randn(1, C, H, W, D, generator=g).to(dev)
f2 = torch.randn(1, C, H, W, D, generator=g).to(dev)
coords = (dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu")) +
          (torch.rand(1, 3, H, W, D, generator=g) * 4 - 2)).to(dev)
dt = ops.dtype_code("bf16")
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
gout = torch.randn(1, L * (2 * R + 1) ** 3, H * W * D, device=dev)
cf = coords.reshape(1, 3, -1).contiguous()
for _ in range(a.reps):
    ops.corr_backward(q, t, cf, gout, C, H, W, D, L, R, bool(a.legacy), dt)
torch.cuda.synchronize()
print("ok")
