#!/usr/bin/env python3
"""Time dvc_corr_backward (HIP events, median of --reps calls after warmup) on the config #3 shape and save
its two gradients, so that builds of libdvccorr (DVCCORR_LIB) can be compared for speed and results:

    DVCCORR_LIB=raft-dvc_amd/dvccorr/libdvccorr_base.so python tools/ab_bwd.py --save gpurun_out/bwd_base.pt
    python tools/ab_bwd.py --save gpurun_out/bwd_new.pt --compare gpurun_out/bwd_base.pt
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
from dvccorr import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=32)
ap.add_argument("--channels", type=int, default=128)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--save", default="")
ap.add_argument("--compare", default="")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, C, L, R = a.size, a.channels, 4, 4
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
c = (torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
     + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
dt = ops.dtype_code(a.precision)
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
gout = torch.randn(1, L * (2 * R + 1) ** 3, S ** 3, generator=g).to(dev)
cf = c.reshape(1, 3, -1).contiguous()
for _ in range(3):
    d1, d2 = ops.corr_backward(q, t, cf, gout, C, S, S, S, L, R, False, dt)
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    d1, d2 = ops.corr_backward(q, t, cf, gout, C, S, S, S, L, R, False, dt)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
d1b, d2b = ops.corr_backward(q, t, cf, gout, C, S, S, S, L, R, False, dt)
torch.cuda.synchronize()
rep = bool(torch.equal(d1, d1b) and torch.equal(d2, d2b))
print(f"lib={os.path.basename(os.environ.get('DVCCORR_LIB', 'libdvccorr.so'))} size={S} C={C} {a.precision} "
      f"backward median {statistics.median(ts):.4f} ms min {min(ts):.4f} repeatable={rep}")
if a.save:
    torch.save({"d1": d1.cpu(), "d2": d2.cpu()}, a.save)
if a.compare:
    ref = torch.load(a.compare, weights_only=True)
    for k, v in (("d1", d1), ("d2", d2)):
        r = ref[k]
        err = ((v.cpu() - r).abs().max() / r.abs().max()).item()
        print(f"  {k}: max|diff|/max|ref| = {err:.3e} bitwise={torch.equal(v.cpu(), r)}")
