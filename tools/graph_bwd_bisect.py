"""Capture dvc_corr_backward in a HIP graph under dvc_set_tuning knob sets and compare the replay with eager."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import prng  # noqa: E402
from dvccorr import _lib, ops  # noqa: E402

DEV = torch.device("cuda:0")
S, C, L, r = 16, 64, 4, 4
f1 = torch.from_numpy(prng.normal(950, (1, C, S, S, S))).to(DEV)
f2 = torch.from_numpy(prng.normal(951, (1, C, S, S, S))).to(DEV)
coords = torch.from_numpy(prng.flow_coords(952, 1, S, S, S, 2.0)).to(DEV).reshape(1, 3, -1)
for prec in ("bf16", "fp32"):
    for knobs in ({}, {"bwd_side": 0}, {"bwd_side": 0, "bwd_sort": 0}, {"bwd_side": 0, "bwd_dense": 0},
                  {"bwd_side": 0, "bwd_sort": 0, "bwd_dense": 0}, {"bwd_side": 0, "bwd_mfma": 0}):
        for k, v in knobs.items():
            _lib.set_tuning(k, v)
        G = torch.from_numpy(prng.normal(953, (1, L * (2 * r + 1) ** 3, S ** 3))).to(DEV)
        dt = ops.dtype_code(prec)
        q = ops.pack_queries(f1.reshape(1, C, -1), dt)
        t = ops.pack_targets(f2, L, dt)
        run = lambda g: ops.corr_backward(q, t, coords, g, C, S, S, S, L, r, False, dt)   # noqa: E731
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            run(G)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g1, g2 = run(G)
        graph.replay()
        torch.cuda.synchronize()
        a1, a2 = g1.clone(), g2.clone()
        G.copy_(torch.from_numpy(prng.normal(954, tuple(G.shape))).to(DEV))
        graph.replay()
        torch.cuda.synchronize()
        e1, e2 = run(G)
        torch.cuda.synchronize()
        print(prec, knobs, "same-G replay finite:", bool(torch.isfinite(a2).all()),
              "new-G replay == eager:", torch.equal(g1, e1), torch.equal(g2, e2),
              "max|d2 diff|", float((g2 - e2).abs().max()), flush=True)
        for k in knobs:
            _lib.set_tuning(k, 1)
