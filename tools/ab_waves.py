#!/usr/bin/env python3
"""k_lookup_tile wave layout A/B (dvc_set_tuning lookup_waves 0 | 4): three 3-column waves vs four balanced
waves (3 + 2 + 2 + 2 columns) per workgroup.  Bitwise equality and HIP-event timing (median), on config #3
and on one rank's H-slab of it (--shard-of N), bf16 and fp32 pyramids."""
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
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--shards", default="1,8,4,2")
ap.add_argument("--precisions", default="bf16,fp32")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = 32, 128, 4, 4
g = torch.Generator(device="cpu").manual_seed(5)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
base = torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
coords_full = base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)
res = {}
with torch.no_grad():
    for prec in a.precisions.split(","):
        dt = ops.dtype_code(prec)
        t = ops.pack_targets(f2, L, dt)
        for n in map(int, a.shards.split(",")):
            h0, h1 = slab_bounds(S, n, 0)
            q = ops.pack_queries(f1[:, :, h0:h1].reshape(1, C, -1), dt)
            corr = ops.build(q, t, C, S, S, S, L, dt, dt)
            cf = coords_full[:, :, h0:h1].contiguous().reshape(1, 3, -1).to(dev)
            ref, times = None, {}
            for rnd in range(2):
                for w in (0, 4):
                    _lib.set_tuning("lookup_waves", w)
                    out = ops.lookup(corr, cf, S, S, S, L, R, False, dt)
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = out.clone()
                    elif rnd == 0:
                        print(f"{prec} shard-of {n} waves {w}: bitwise equal {torch.equal(out, ref)}", flush=True)
                        assert torch.equal(out, ref)
                    for _ in range(a.reps):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        ops.lookup(corr, cf, S, S, S, L, R, False, dt, out=out)
                        e1.record()
                        e1.synchronize()
                        times.setdefault(w, []).append(e0.elapsed_time(e1))
            res[f"{prec}_shard{n}"] = {w: round(1e3 * statistics.median(v), 1) for w, v in times.items()}
            del corr, q
            torch.cuda.empty_cache()
_lib.set_tuning("lookup_waves", 0)
print(json.dumps({"median_us": res}))
