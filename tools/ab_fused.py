#!/usr/bin/env python3
"""A/B timing of the fused lookup kernels (dvc_set_tuning fused_variant), HIP events on the launch stream,
interleaved rounds, median per variant.  Prints one JSON line.

    python tools/ab_fused.py --size 128 --levels 2 --variants 1,2,3
"""
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
from dvccorr import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--radius", type=int, default=4)
ap.add_argument("--max-flow", type=float, default=2.0)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="1,2,3")
ap.add_argument("--check", action="store_true", help="compare every variant's output with the first one")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, 128, a.levels, a.radius
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
c = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) +
     (torch.rand(1, 3, S, S, S, generator=g) * 2 - 1) * a.max_flow).to(dev)
blk = dvccorr.CorrBlockFused(f1, f2, L, R, precision="bf16")
variants = a.variants.split(",")   # "V" or "V:aN" (fused_ablate N, diagnostics)


def select(v):
    parts = v.split(":a")
    _lib.set_tuning("fused_variant", int(parts[0]))
    _lib.set_tuning("fused_ablate", int(parts[1]) if len(parts) > 1 else 0)


times = {v: [] for v in variants}
first = None
stream = torch.cuda.current_stream(dev)
with torch.no_grad():
    for rnd in range(a.rounds):
        for v in variants:
            select(v)
            out = blk(c)
            if a.check and rnd == 0:
                torch.cuda.synchronize()
                if ":a" in v:
                    pass
                elif first is None:
                    first = out.clone()
                else:
                    print(f"variant {v}: equal={torch.equal(out, first)} "
                          f"maxdiff={float((out - first).abs().max()):.3e}", flush=True)
            del out
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                o = blk(c)
                e1.record(stream)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1))
                del o
select("2")
print(json.dumps({"size": S, "levels": L, "radius": R, "max_flow": a.max_flow,
                  "median_ms": {v: round(statistics.median(t), 4) for v, t in times.items()},
                  "min_ms": {v: round(min(t), 4) for v, t in times.items()}}), flush=True)
