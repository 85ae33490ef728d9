"""Pins the closed-loop harness (tests/raftdvc_loop.py) on CPU: with the reference-equivalent correlation
(oracle/torch_cpu.py, bit-identical to corr.py) and the reference's own upflow ops, the 12-iteration loop
reproduces the reference RAFTDVC's final low-res flow (tests/golden/epe_1_8.npz) -- so the GPU test's EPE
measures dvccorr alone."""
from __future__ import annotations

import numpy as np
import torch

import raftdvc_loop as rl
from conftest import load_golden
from oracle import torch_cpu


def test_harness_reproduces_reference_flow():
    g = load_golden("epe_1_8.npz")
    p = rl.load_params("cpu")
    f0, f1 = torch.from_numpy(g["fmap0"]), torch.from_numpy(g["fmap1"])
    B, _, h, w, d = f0.shape
    ax = [torch.arange(s, dtype=torch.float32) for s in (h, w, d)]
    coords0 = torch.stack(torch.meshgrid(*ax, indexing="ij"))[None].expand(B, 3, h, w, d).contiguous()
    T = tuple(int(v) for v in g["target_shape"])
    with torch.no_grad():
        flow_lo, flow_up, deltas = rl.refine(
            lambda c: torch_cpu.corr_lookup(f0, f1, c, 4, 4, False),
            lambda c, dl: rl.reference_tail(c, dl, coords0, T),
            p, torch.from_numpy(g["net0"]), torch.from_numpy(g["context"]), coords0, 12, T)
    e = rl.epe(flow_lo, g["flow_lo"])
    assert e < 1e-6, e
    for i, dl in enumerate(deltas):
        assert np.abs(dl.numpy() - g["delta"][i]).max() < 1e-5, i
    up = flow_up.double().numpy()
    cs = g["flow_up_checksum"]
    assert abs(up.sum() - cs[0]) <= 1e-4 * cs[1] and abs(np.abs(up).max() - cs[3]) <= 1e-5 * cs[3]
