#!/usr/bin/env python3
"""A/B timing of kernel variants in one process (interleaved rounds, HIP events).

    python tools/ab_kernels.py [--size 32] [--precision bf16] [--rounds 5] [--reps 12]
Prints per-variant median/min lookup ms and build ms, plus correctness deltas
between variants (must be ~0)."""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
# the diagnostics knobs (ablations, traces, store policies) live in libdvccorr_diag.so (make -C raft-dvc_amd/csrc diag)
os.environ.setdefault("DVCCORR_LIB", os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr_diag.so"))
import dvccorr  # noqa: E402
from dvccorr import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--radius", type=int, default=4)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=12)
ap.add_argument("--variants", default="0,2", help="comma list; a variant may carry knobs: 2:lookup_nt=1")
ap.add_argument("--ablate", default="", help="comma list of lookup_ablate values to time (diagnostics)")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, L, R = a.size, a.levels, a.radius
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
c = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) +
     (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
variants = a.variants.split(",")


def apply(v):
    parts = v.split(":")
    for k, d in (("lookup_nt", 1), ("lookup_order", 1), ("lookup_ldpol", 0)):
        _lib.set_tuning(k, d)
    _lib.set_tuning("lookup_variant", int(parts[0]))
    for kv in parts[1:]:
        k, val = kv.split("=")
        _lib.set_tuning(k, int(val))

res = {v: [] for v in variants}
bres = []
outs = {}
with torch.no_grad():
    for rnd in range(a.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        blk = dvccorr.CorrBlock(f1, f2, L, R, precision=a.precision)
        e1.record()
        torch.cuda.synchronize()
        bres.append(e0.elapsed_time(e1))
        for v in variants:
            apply(v)
            out = blk(c)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                out = blk(c)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.reps)
            outs[v] = out
if a.ablate:
    abl = {}
    with torch.no_grad():
        for v in [int(x) for x in a.ablate.split(",")]:
            apply(variants[0])
            _lib.set_tuning("lookup_ablate", v)
            ts = []
            for _ in range(a.rounds):
                blk(c)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.reps):
                    blk(c)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / a.reps)
            abl[v] = statistics.median(ts)
        _lib.set_tuning("lookup_ablate", 0)
    print(json.dumps({"ablate_ms": abl}))
base = outs[variants[0]]
summary = {"size": S, "precision": a.precision, "build_ms_median": statistics.median(bres),
           "variants": {v: {"median_ms": statistics.median(t), "min_ms": min(t),
                            "max_abs_diff_vs_first": float((outs[v] - base).abs().max())} for v, t in res.items()}}
print(json.dumps(summary))
