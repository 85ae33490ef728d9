#!/usr/bin/env python3
"""Minimal workload for rocprofv3 passes over the backward (dvc_corr_backward) at config #3's shape."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
from dvccorr import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
c = (torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
     + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
dt = ops.dtype_code(a.precision)
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
gout = torch.randn(1, L * (2 * R + 1) ** 3, S ** 3, generator=g).to(dev)
cf = c.reshape(1, 3, -1).contiguous()
for _ in range(a.reps):
    ops.corr_backward(q, t, cf, gout, C, S, S, S, L, R, False, dt)
torch.cuda.synchronize()
print("ok")
