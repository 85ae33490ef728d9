#!/usr/bin/env python3
"""Ablation timings of the convc1-fused on-the-fly lookup (dvc_corr_lookup_fused_proj) at config #5
(128^3 x 128 fmaps, L=2, r=4, coords = identity + U(-2, 2)).  Diagnostics only: the fused_ablate bits
skip parts of k_fused_proj (1 phase 1, 2 producers, 4 convc1 MFMA, 8 window writes, 16 target loads)."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
# the diagnostics knobs (ablations, traces, store policies) live in libdvccorr_diag.so (make -C raft-dvc_amd/csrc diag)
os.environ.setdefault("DVCCORR_LIB", os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr_diag.so"))
import dvccorr  # noqa: E402
from dvccorr import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=128)
ap.add_argument("--levels", type=int, default=2)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--ablate", default="0,1,3,7,2,4,6,8,16,24")
ap.add_argument("--knobs", default="", help="';'-separated knob settings (key=value,...) timed at ablate 0 after the "
                                            "ablations, outputs compared bitwise with the default's")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, L = a.size, a.levels
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
c = (dvccorr.coords_grid_3d(1, S, S, S, torch.device("cpu")) + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
K = L * 729
w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
b = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev)
res = {}
with torch.no_grad():
    blk = dvccorr.CorrBlockFused(f1, f2, L, 4, precision="bf16")
    for v in [int(x) for x in a.ablate.split(",")]:
        _lib.set_tuning("fused_ablate", v)
        blk.lookup_convc1(c, w, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            blk.lookup_convc1(c, w, b)
        e1.record()
        torch.cuda.synchronize()
        res[v] = round(e0.elapsed_time(e1) / a.reps, 3)
        print(f"ablate {v}: {res[v]} ms per lookup_convc1", flush=True)
    _lib.set_tuning("fused_ablate", 0)
    ref = blk.lookup_convc1(c, w, b).clone()
    for setting in [x for x in a.knobs.split(";") if x]:
        kv = [x.split("=") for x in setting.split(",")]
        for k, v in kv:
            _lib.set_tuning(k, int(v))
        o = blk.lookup_convc1(c, w, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            blk.lookup_convc1(c, w, b)
        e1.record()
        torch.cuda.synchronize()
        res[setting] = round(e0.elapsed_time(e1) / a.reps, 3)
        print(f"{setting}: {res[setting]} ms per lookup_convc1, bitwise equal to default: {torch.equal(o, ref)}",
              flush=True)
        for k, v in kv:
            _lib.set_tuning(k, 0)
print(json.dumps({"size": S, "levels": L, "ms": res}))
