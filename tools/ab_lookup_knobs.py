#!/usr/bin/env python3
"""HIP-event timing (median) of the config #3 lookup under dvc_set_tuning knob sets, interleaved rounds.
Diagnostics only: ablation knobs (lookup_ablate) produce invalid outputs.

    python tools/ab_lookup_knobs.py "lookup_waves=0" "lookup_waves=4" "lookup_waves=0,lookup_ablate=4"
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
# the diagnostics knobs (ablations, traces, store policies) live in libdvccorr_diag.so (make -C raft-dvc_amd/csrc diag)
os.environ.setdefault("DVCCORR_LIB", os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr_diag.so"))
from dvccorr import _lib, ops  # noqa: E402

DEFAULTS = {"lookup_waves": 4, "lookup_ablate": 0}
sets = sys.argv[1:] or ["lookup_waves=4"]
dev = torch.device("cuda:0")
S, C, L, R = 32, 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
base = torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
cf = (base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).reshape(1, 3, -1).to(dev)
dt = ops.dtype_code("bf16")
corr = ops.build(ops.pack_queries(f1.reshape(1, C, -1), dt), ops.pack_targets(f2, L, dt), C, S, S, S, L, dt, dt)
out = ops.lookup(corr, cf, S, S, S, L, R, False, dt)
times = {k: [] for k in sets}


def apply(ks):
    kv = dict(DEFAULTS)
    for item in filter(None, ks.split(",")):
        k, v = item.split("=")
        kv[k] = int(v)
    for k, v in kv.items():
        _lib.set_tuning(k, v)


with torch.no_grad():
    for rnd in range(3):
        for ks in sets:
            apply(ks)
            for _ in range(3):
                ops.lookup(corr, cf, S, S, S, L, R, False, dt, out=out)
            for _ in range(15):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.lookup(corr, cf, S, S, S, L, R, False, dt, out=out)
                e1.record()
                e1.synchronize()
                times[ks].append(e0.elapsed_time(e1))
apply("")
print(json.dumps({"median_us": {k: round(1e3 * statistics.median(v), 1) for k, v in times.items()}}))
