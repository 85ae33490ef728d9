#!/usr/bin/env python3
"""Row-split variants of the slab lookup (dvc_set_tuning split_ach 0 | 2 | 3 | 5): bitwise equality with the
default and HIP-event timing, on one rank's H-slab of config #3 (--shard-of N)."""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
from dvccorr import _lib, ops  # noqa: E402
from dvccorr.sharded import slab_bounds  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shard-of", type=int, default=8)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = 32, 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
h0, h1 = slab_bounds(S, a.shard_of, 0)
base = torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
coords = (base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2))[:, :, h0:h1].contiguous().to(dev)
dt = ops.dtype_code("bf16")
q = ops.pack_queries(f1[:, :, h0:h1].reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
corr = ops.build(q, t, C, S, S, S, L, dt, dt)
cf = coords.reshape(1, 3, -1)
res, ref = {}, None
with torch.no_grad():
    for rnd in range(2):
        for ach in (3, 0, 2, 5):
            _lib.set_tuning("split_ach", ach)
            out = ops.lookup(corr, cf, S, S, S, L, R, False, dt)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif rnd == 0:
                print(f"split_ach {ach}: bitwise equal {torch.equal(out, ref)}", flush=True)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.lookup(corr, cf, S, S, S, L, R, False, dt, out=out)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            res.setdefault(ach, []).extend(ts)
_lib.set_tuning("split_ach", 3)
print(json.dumps({"shard_of": a.shard_of, "rows": h1 - h0, "median_us": {k: round(1e3 * statistics.median(v), 1)
                                                                          for k, v in res.items()}}))
