#!/usr/bin/env python3
"""A/B of the default lookup path (CorrBlock, bricked bf16 pyramid) under dvc_set_tuning knob sets:
HIP-event medians over interleaved rounds, outputs compared bit for bit with the first set.

    python tools/ab_lookup.py [--size 32] [--precision bf16] [--convc1] "" "lookup_stpol=16" ...
    DVCCORR_LIB=.../libdvccorr_base.so python tools/ab_lookup.py ...     (another build of the same ABI)

Diagnostics only: ablation knobs make outputs invalid (reported, not asserted)."""
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
ap.add_argument("sets", nargs="*", default=[""])
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--convc1", action="store_true")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--calls", type=int, default=15)
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, 128, a.levels, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
base = torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
coords = (base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
K = L * (2 * R + 1) ** 3
w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
b = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev)


def apply(ks, reset=False):
    for item in filter(None, ks.split(",")):
        k, v = item.split("=")
        # (reset to the library defaults, not 0: lookup_waves is 4, split_tiles 1024, lookup_stpol -1)
        _lib.set_tuning(k, {"lookup_stpol": -1, "lookup_waves": 4, "split_tiles": 1024, "split_ach": 5,
                            "lookup_variant": 2, "lookup_nt": 1, "lookup_order": 1}.get(k, 0) if reset else int(v))


with torch.no_grad():
    blk = dvccorr.CorrBlock(f1, f2, L, R, precision=a.precision)
    call = (lambda: blk.lookup_convc1(coords, w, b)) if a.convc1 else (lambda: blk(coords))
    times = {k: [] for k in a.sets}
    outs = {}
    for rnd in range(a.rounds):
        for ks in a.sets:
            apply(ks)
            for _ in range(3):
                o = call()
            if rnd == 0:
                outs[ks] = o.clone()
            for _ in range(a.calls):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                call()
                e1.record()
                torch.cuda.synchronize()
                times[ks].append(e0.elapsed_time(e1) * 1e3)
            apply(ks, reset=True)
    ref = outs[a.sets[0]]
    res = {"lib": os.path.basename(_lib.LIB_PATH), "size": S, "precision": a.precision, "convc1": a.convc1}
    for ks in a.sets:
        res[ks or "default"] = {"median_us": round(statistics.median(times[ks]), 2),
                                "min_us": round(min(times[ks]), 2),
                                "bitwise_equal_first": bool(torch.equal(outs[ks], ref))}
    print(json.dumps(res))
