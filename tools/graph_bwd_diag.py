"""dvc_corr_backward in a HIP graph with a caller-owned workspace (poisoned before capture): does the replay zero the
256-byte guard (the captured hipMemsetAsync), and do the replayed gradients equal eager ones?"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import prng  # noqa: E402
from dvccorr import _lib, ops  # noqa: E402
from dvccorr.ops import _ptr, _stream, lib  # noqa: E402

DEV = torch.device("cuda:0")
S, C, L, r = 16, 64, 4, 4
B, Nq = 1, S ** 3
f1 = torch.from_numpy(prng.normal(950, (1, C, S, S, S))).to(DEV)
f2 = torch.from_numpy(prng.normal(951, (1, C, S, S, S))).to(DEV)
coords = torch.from_numpy(prng.flow_coords(952, 1, S, S, S, 2.0)).to(DEV).reshape(1, 3, -1).contiguous()
G = torch.from_numpy(prng.normal(953, (1, L * (2 * r + 1) ** 3, S ** 3))).to(DEV).contiguous()
dt = ops.dtype_code("bf16")
q = ops.pack_queries(f1.reshape(1, C, -1), dt)
t = ops.pack_targets(f2, L, dt)
nws = lib().dvc_corr_backward_workspace_bytes_dtype(B, Nq, C, S, S, S, L, r, dt)
ws = torch.full((nws // 4 + 64,), float("nan"), device=DEV)
d1 = torch.empty((B, C, Nq), device=DEV)
d2 = torch.empty((B, C, S, S, S), device=DEV)


def run(wsb):
    ops.check(lib().dvc_corr_backward(_ptr(q), _ptr(t), _ptr(coords), _ptr(G), _ptr(d1), _ptr(d2), _ptr(wsb), B, Nq, C,
                                      S, S, S, L, r, 0, dt, _stream(q)), "bwd")


e1, e2 = ops.corr_backward(q, t, coords, G, C, S, S, S, L, r, False, dt)
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.graph(graph, stream=s):
    run(ws)
torch.cuda.synchronize()
print("after capture: guard finite?", bool(torch.isfinite(ws[:64]).all()), "d2 == eager?", torch.equal(d2, e2))
graph.replay()
torch.cuda.synchronize()
print("after replay 1: guard zero?", bool((ws[:64] == 0).all()), "d1 == eager", torch.equal(d1, e1),
      "d2 == eager", torch.equal(d2, e2), "max diff", float((d2 - e2).abs().max()))
ws.fill_(float("nan"))
graph.replay()
torch.cuda.synchronize()
print("after poison + replay 2: guard zero?", bool((ws[:64] == 0).all()), "d2 == eager", torch.equal(d2, e2),
      "max diff", float((d2 - e2).abs().max()))
_lib.set_tuning("bwd_side", 0)
ws.fill_(float("nan"))
run(ws)
torch.cuda.synchronize()
print("eager caller-ws (poisoned): d2 == eager", torch.equal(d2, e2), "guard zero?", bool((ws[:64] == 0).all()))
