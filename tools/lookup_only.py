#!/usr/bin/env python3
"""Minimal workload for rocprofv3 counter passes: one build + `reps` lookups."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
import dvccorr  # noqa: E402
from dvccorr import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--impl", default="materialised")
ap.add_argument("--tune", default="", help="comma list key=value of dvc_set_tuning knobs")
ap.add_argument("--convc1", action="store_true", help="lookup_convc1 (convc1 fused) instead of the lookup")
ap.add_argument("--shard-of", type=int, default=1,
                help="rank 0's H slab of an N-way split (bench.py --shard-of): its rows against the whole fmap2")
ap.add_argument("--build", default="gemm", choices=["gemm", "pool"],
                help="materialised pyramid: GEMM against pooled targets (default) or level-0 GEMM + k_corr_pool")
a = ap.parse_args()
_lib.set_tuning("lookup_variant", a.variant)
for kv in filter(None, a.tune.split(",")):
    k, v = kv.split("=")
    _lib.set_tuning(k, int(v))
dev = torch.device("cuda:0")
S = a.size
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
c = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
with torch.no_grad():
    if a.shard_of > 1:
        from dvccorr.sharded import HipRows
        h1 = S // a.shard_of
        blk = HipRows(f1[:, :, :h1].reshape(1, 128, -1).contiguous(), f2, a.levels, 4, False, a.precision, a.impl)
        c = c[:, :, :h1].reshape(1, 3, -1).contiguous()
    else:
        cls = dvccorr.CorrBlock if a.impl == "materialised" else dvccorr.CorrBlockFused
        # (the walk variants read the linear layout only)
        kw = {"build": a.build, "bricked": None if a.variant == 2 else False} if a.impl == "materialised" else {}
        blk = cls(f1, f2, a.levels, 4, precision=a.precision, **kw)
    K = a.levels * 729
    w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
    bias = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev)
    for _ in range(a.reps):
        out = blk.lookup_convc1(c, w, bias) if a.convc1 else (blk.lookup(c) if a.shard_of > 1 else blk(c))
torch.cuda.synchronize()
print("ok", float(out.abs().sum()))
