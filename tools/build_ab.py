#!/usr/bin/env python3
"""Time the build kernel alone (HIP events) under tuning knobs / ablations, and compare its pyramid with the
first setting's (bitwise flag + max relative difference).

    python tools/build_ab.py [--size 32] [--precision bf16|fp16|fp32] [--reps 10] \
        [--knobs "build_f32_variant=0;build_ablate=1"]

Knobs are reset to 0 after their setting (build_f32_variant / build_variant default to 1: pass them explicitly
in every setting that needs a non-default value)."""
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
ap.add_argument("--channels", type=int, default=128)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--knobs", default="", help="';'-separated settings, each a ','-list of key=value")
a = ap.parse_args()
dev = torch.device("cuda:0")
S, L, C = a.size, a.levels, a.channels
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, C, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, C, S, S, S, generator=g).to(dev)
dt = ops.dtype_code(a.precision)
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
lay = dvccorr.layout(S, S, S, L, C)
esz = 4 if a.precision == "fp32" else 2
nbytes = S ** 3 * sum(h * w * d for h, w, d in lay.levels()) * esz
flops = 2.0 * S ** 6 * C
res = {"size": S, "precision": a.precision}
first = None
defaults = {"build_f32_variant": 2, "build_variant": 1}
for setting in [""] + [x for x in a.knobs.split(";") if x]:
    kv = [x.split("=") for x in setting.split(",") if x]
    for k, v in kv:
        _lib.set_tuning(k, int(v))
    out = ops.alloc_corr(1, S ** 3, lay.row_stride, dt, dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for r in range(a.reps + 2):
        e0.record()
        ops.build(q, t, C, S, S, S, L, dt, dt, out=out)
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    for k, v in kv:
        _lib.set_tuning(k, defaults.get(k, 0))
    m = statistics.median(ts)
    o = out.float()
    if first is None:
        first = o
    diff = float((o - first).abs().max() / first.abs().max())
    res[setting or "default"] = {"median_ms": round(m, 4), "min_ms": round(min(ts), 4),
                                 "GB/s": round(nbytes / (m * 1e-3) / 1e9, 1),
                                 "TFLOP/s": round(flops / (m * 1e-3) / 1e12, 1),
                                 "bitwise_equal_first": bool(torch.equal(o, first)), "max_rel_diff_first": diff}
    del out, o
    torch.cuda.empty_cache()
print(json.dumps(res))
