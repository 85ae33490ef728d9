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
ap.add_argument("--shape", default="", help="H,W,D (default: size^3)")
ap.add_argument("--levels", type=int, default=4)
ap.add_argument("--radius", type=int, default=4)
ap.add_argument("--channels", type=int, default=128)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--save", default="")
ap.add_argument("--compare", default="")
ap.add_argument("--tune", default="", help="comma list key=value of dvc_set_tuning knobs (e.g. bwd_g16=0)")
a = ap.parse_args()
for kv in filter(None, a.tune.split(",")):
    k, v = kv.split("=")
    ops._lib.set_tuning(k, int(v))
dev = torch.device("cuda:0")
S, C, L, R = a.size, a.channels, a.levels, a.radius
H, W, D = (int(v) for v in a.shape.split(",")) if a.shape else (S, S, S)
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, C, H, W, D, generator=g).to(dev)
f2 = torch.randn(1, C, H, W, D, generator=g).to(dev)
c = (torch.stack(torch.meshgrid(*[torch.arange(n, dtype=torch.float32) for n in (H, W, D)], indexing="ij"))[None]
     + (torch.rand(1, 3, H, W, D, generator=g) * 4 - 2)).to(dev)
dt = ops.dtype_code(a.precision)
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
gout = torch.randn(1, L * (2 * R + 1) ** 3, H * W * D, generator=g).to(dev)
cf = c.reshape(1, 3, -1).contiguous()
for _ in range(3):
    d1, d2 = ops.corr_backward(q, t, cf, gout, C, H, W, D, L, R, False, dt)
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    d1, d2 = ops.corr_backward(q, t, cf, gout, C, H, W, D, L, R, False, dt)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
d1b, d2b = ops.corr_backward(q, t, cf, gout, C, H, W, D, L, R, False, dt)
torch.cuda.synchronize()
rep = bool(torch.equal(d1, d1b) and torch.equal(d2, d2b))
print(f"lib={os.path.basename(os.environ.get('DVCCORR_LIB', 'libdvccorr.so'))} tune={a.tune} size={S} C={C} {a.precision} "
      f"backward median {statistics.median(ts):.4f} ms min {min(ts):.4f} repeatable={rep}")
if a.save:
    torch.save({"d1": d1.cpu(), "d2": d2.cpu()}, a.save)
if a.compare:
    ref = torch.load(a.compare, weights_only=True)
    for k, v in (("d1", d1), ("d2", d2)):
        r = ref[k]
        err = ((v.cpu() - r).abs().max() / r.abs().max()).item()
        print(f"  {k}: max|diff|/max|ref| = {err:.3e} bitwise={torch.equal(v.cpu(), r)}")
        if k == "d1" and err > 1e-3:   # where: per 32-channel tile, per query z
            dd = (v.cpu() - r).abs()[0]
            print("    per 32-ch tile:", [round(float(dd[i:i + 32].max()), 4) for i in range(0, dd.shape[0], 32)])
            print("    per query z:", [round(float(x), 4) for x in dd.reshape(dd.shape[0], H, W, D).amax((0, 1, 2))])
