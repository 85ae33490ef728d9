#!/usr/bin/env python3
"""Workload for a rocprofv3 kernel trace of the legacy non-cubic lookup (tools/bench_legacy.py's shape): `reps` lookups."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
import dvccorr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="32,32,16")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--fused", action="store_true", help="the on-the-fly block instead of the materialised one")
a = ap.parse_args()
H, W, D = (int(x) for x in a.shape.split(","))
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(11)
f1 = torch.randn(1, 128, H, W, D, generator=g).to(dev)
f2 = torch.randn(1, 128, H, W, D, generator=g).to(dev)
c = (dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu")) + (torch.rand(1, 3, H, W, D, generator=g) * 4 - 2)).to(dev)
with torch.no_grad():
    cls = dvccorr.CorrBlockFused if a.fused else dvccorr.CorrBlock
    blk = cls(f1, f2, 4, 4, True, precision="bf16")
    for _ in range(a.reps):
        out = blk(c)
torch.cuda.synchronize()
print("ok")
