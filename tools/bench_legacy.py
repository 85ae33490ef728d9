#!/usr/bin/env python3
"""Legacy sampler convention on a non-cubic volume (verdict r5 "missing" #3): the reference's legacy_wd_swap
(corr.py:49-52) samples a W != D level on a stretched lattice, so those levels take the walk / generic kernels
(lookup, on-the-fly, unfused convc1) while the fixed convention keeps the tile / box kernels.  Times both conventions
on the same (H, W, D) fmap pair, HIP events on the launch stream, medians; one JSON line.

    python tools/bench_legacy.py --shape 32,32,16
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
import dvccorr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="32,32,16", help="fmap H,W,D (W != D: the legacy levels go generic)")
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--radius", type=int, default=4)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--precision", default="bf16")
a = ap.parse_args()
H, W, D = (int(x) for x in a.shape.split(","))
dev = torch.device("cuda:0")
C, L, R = 128, a.levels, a.radius
g = torch.Generator(device="cpu").manual_seed(11)
f1 = torch.randn(1, C, H, W, D, generator=g).to(dev)
f2 = torch.randn(1, C, H, W, D, generator=g).to(dev)
coords = (dvccorr.coords_grid_3d(1, H, W, D, torch.device("cpu")) +
          (torch.rand(1, 3, H, W, D, generator=g) * 4 - 2)).to(dev)
K = L * (2 * R + 1) ** 3
wc = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
bc = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev)
stream = torch.cuda.current_stream(dev)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return round(statistics.median(ts), 4)


out = {"shape": [H, W, D], "levels": L, "radius": R, "precision": a.precision, "query_voxels": H * W * D,
       "what": "median ms per call, HIP events; build = CorrBlock construction (pack + GEMM pyramid)"}
with torch.no_grad():
    for legacy in (False, True):
        key = "legacy" if legacy else "fixed"
        r = {}
        r["build_ms"] = timed(lambda: dvccorr.CorrBlock(f1, f2, L, R, legacy, precision=a.precision))
        blk = dvccorr.CorrBlock(f1, f2, L, R, legacy, precision=a.precision)
        r["lookup_ms"] = timed(lambda: blk(coords))
        r["lookup_convc1_ms"] = timed(lambda: blk.lookup_convc1(coords, wc, bc))
        fb = dvccorr.CorrBlockFused(f1, f2, L, R, legacy, precision=a.precision)
        r["fused_lookup_ms"] = timed(lambda: fb(coords))
        # the training backward (dvc_corr_backward: d fmap1, d fmap2 of one lookup) on these inputs
        from dvccorr import ops
        dt = ops.dtype_code(a.precision)
        q = ops.pack_queries(f1.reshape(1, C, -1), dt)
        t = ops.pack_targets(f2, L, dt)
        gout = torch.randn(1, L * (2 * R + 1) ** 3, H * W * D, device=dev)
        cf = coords.reshape(1, 3, -1).contiguous()
        r["backward_ms"] = timed(lambda: ops.corr_backward(q, t, cf, gout, C, H, W, D, L, R, legacy, dt))
        if legacy:   # same values through both impls (the generic kernels of each)
            d = (blk(coords) - fb(coords)).abs().max().item()
            r["materialised_vs_fused_maxdiff"] = d
        out[key] = r
        del blk, fb
        torch.cuda.empty_cache()
out["lookup_legacy_over_fixed"] = round(out["legacy"]["lookup_ms"] / out["fixed"]["lookup_ms"], 2)
print(json.dumps(out), flush=True)
