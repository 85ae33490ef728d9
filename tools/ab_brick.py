#!/usr/bin/env python3
"""A/B of the DVC_BRICKED pyramid layout (levels with >= 64-byte z-rows in (1, 8, 8) bricks) against the linear
layout: the same CorrBlock built both ways (bricked=False vs the default), bitwise-equal lookups, HIP-event
medians of the lookup and of the convc1-fused lookup, interleaved rounds.

    python tools/ab_brick.py [--size 32] [--precisions bf16,fp32]
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
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--reps", type=int, default=15)
ap.add_argument("--precisions", default="bf16,fp32")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, 128, a.levels, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
c = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
K = L * (2 * R + 1) ** 3
w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
bias = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev)
res = {}
with torch.no_grad():
    for prec in a.precisions.split(","):
        lin = dvccorr.CorrBlock(f1, f2, L, R, precision=prec, bricked=False)
        brk = dvccorr.CorrBlock(f1, f2, L, R, precision=prec)
        runs = {"linear": lambda: lin(c), "bricked": lambda: brk(c)}
        if prec == "bf16":
            runs.update({"convc1_linear": lambda: lin.lookup_convc1(c, w, bias),
                         "convc1_bricked": lambda: brk.lookup_convc1(c, w, bias)})
        outs, times = {}, {k: [] for k in runs}
        for rnd in range(3):
            for k, fn in runs.items():
                o = fn()
                torch.cuda.synchronize()
                outs.setdefault(k, o.clone())
                for _ in range(a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    e1.synchronize()
                    times[k].append(e0.elapsed_time(e1))
        eq = [torch.equal(outs["linear"], outs["bricked"])]
        if prec == "bf16":
            eq.append(torch.equal(outs["convc1_linear"], outs["convc1_bricked"]))
        print(f"{prec}: bricked levels {bin(dvccorr.ops.bricked_levels(brk._lay))}, bitwise equal {eq}", flush=True)
        res[prec] = {k: round(1e3 * statistics.median(v), 1) for k, v in times.items()}
        res[prec]["equal"] = eq
        del lin, brk
        torch.cuda.empty_cache()
print(json.dumps({"size": S, "levels": L, "median_us": res}))
