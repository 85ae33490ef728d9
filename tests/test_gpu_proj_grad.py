"""GPU parity of the differentiable fused convc1 lookup (dvccorr::lookup_convc1_ad): the Trainer's path
(trainer.py:249-257 runs update.py:246, relu(convc1(corr)), under autograd), where the L*(2r+1)^3-channel lookup
tensor is neither written by the forward nor saved for the backward.

Oracle: fp32 autograd on the CPU through oracle/torch_cpu.py (the reference's corr.py:116-208 restated, pinned by the
grad_* golden vectors) followed by conv3d (update.py:222) and the ReLU.  The ReLU decision is taken from the GPU's
own output (y > 0): where the pre-activation is within the fp16 MFMA's ~1e-3 of zero the two sides may switch a
ReLU differently, which is a discontinuity, not an error of the gradient; the test checks that the decisions agree
on >= 99.5 % of the outputs and then compares the gradients of the same piecewise-linear function.
Shapes: grad_cfg2 (config #2's 16^3, C = 128, L = 4, r = 4, reference-seeded inputs) and a ragged 12x10x16 case.
Tolerances (max|gpu - ref| / max|ref|): bf16 blocks 1e-2, fp16 (AMP) blocks 5e-3, fp32 (materialised, the exact
split convc1) 1e-5.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import prng
from conftest import grad_inputs, load_golden
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
TOL = {"bf16": 1e-2, "fp16": 5e-3, "fp32": 1e-5}


def _case(name):
    if name == "grad_cfg2":
        f1, f2, coords, _G, L, r, legacy = grad_inputs(load_golden("grad_cfg2.npz"))
    else:   # ragged: tiles and sorted groups with partial occupancy, non-cubic levels
        B, C, H, W, D, L, r = 1, 64, 12, 10, 16, 3, 4
        f1 = prng.normal(7101, (B, C, H, W, D))
        f2 = prng.normal(7102, (B, C, H, W, D))
        coords = prng.flow_coords(7103, B, H, W, D, 3.0)
        legacy = False
    B, C, H, W, D = f1.shape
    K = L * (2 * r + 1) ** 3
    w = prng.uniform(7201, (96, K), -K ** -0.5, K ** -0.5)
    b = prng.uniform(7202, (96,), -K ** -0.5, K ** -0.5)
    gy = prng.normal(7203, (B, 96, H, W, D))
    return f1, f2, coords, w, b, gy, L, r, legacy


def _oracle(f1, f2, coords, w, b, gy, mask, L, r, legacy):
    from oracle import torch_cpu
    t1 = torch.from_numpy(np.ascontiguousarray(f1)).requires_grad_(True)
    t2 = torch.from_numpy(np.ascontiguousarray(f2)).requires_grad_(True)
    tw = torch.from_numpy(w).requires_grad_(True)
    tb = torch.from_numpy(b).requires_grad_(True)
    x = torch_cpu.corr_lookup(t1, t2, torch.from_numpy(coords), L, r, legacy)
    pre = torch.nn.functional.conv3d(x, tw.view(96, -1, 1, 1, 1), tb)
    ((pre * torch.from_numpy(mask)) * torch.from_numpy(gy)).sum().backward()
    return pre.detach().numpy(), t1.grad.numpy(), t2.grad.numpy(), tw.grad.numpy(), tb.grad.numpy()


@pytest.mark.parametrize("precision,kind", [("bf16", "gemm"), ("bf16", "fused"), ("fp16", "gemm"), ("fp16", "fused"),
                                            ("fp32", "gemm")])
@pytest.mark.parametrize("case", ["grad_cfg2", "ragged"])
def test_lookup_convc1_grad(case, precision, kind):
    import dvccorr
    f1, f2, coords, w, b, gy, L, r, legacy = _case(case)
    t1 = torch.from_numpy(f1).to(DEV).requires_grad_(True)
    t2 = torch.from_numpy(f2).to(DEV).requires_grad_(True)
    tw = torch.from_numpy(w.reshape(96, -1, 1, 1, 1)).to(DEV).requires_grad_(True)
    tb = torch.from_numpy(b).to(DEV).requires_grad_(True)
    cls = dvccorr.CorrBlock if kind == "gemm" else dvccorr.CorrBlockFused
    blk = cls(t1, t2, L, r, legacy_wd_swap=legacy, precision=precision)

    def _no_composition(*a, **k):
        raise AssertionError("lookup_convc1 took the unfused composition under autograd")
    blk._convc1_composition = _no_composition
    out = blk.lookup_convc1(torch.from_numpy(coords).to(DEV), tw, tb)
    (out * torch.from_numpy(gy).to(DEV)).sum().backward()
    torch.cuda.synchronize()
    y = out.detach().cpu().numpy()
    mask = (y > 0).astype(np.float32)
    pre, r1, r2, rw, rb = _oracle(f1, f2, coords, w, b, gy, mask, L, r, legacy)
    assert np.mean((pre > 0) == (mask > 0)) >= 0.995
    tol = TOL[precision]
    assert orc.rel_err(y, np.maximum(pre, 0.0)) <= tol
    for got, ref, name in ((t1.grad, r1, "fmap1"), (t2.grad, r2, "fmap2"), (tw.grad.view(96, -1), rw, "weight"),
                           (tb.grad, rb, "bias")):
        g = got.detach().cpu().numpy()
        assert np.isfinite(g).all(), name
        e = orc.rel_err(g, ref)
        assert e <= tol, (name, e)


def test_lookup_convc1_grad_weight_only():
    """An inference block (fmaps without grad: bricked pyramid, no packed operands kept) with a trainable convc1:
    dW and db through the recomputed (bricked) lookup, no fmap gradient asked for."""
    import dvccorr
    B, C, H, W, D, L, r, legacy = 1, 32, 8, 8, 32, 2, 4, False    # level 0 with 64-byte z-rows: (1, 8, 8) bricks
    f1 = prng.normal(7301, (B, C, H, W, D))
    f2 = prng.normal(7302, (B, C, H, W, D))
    coords = prng.flow_coords(7303, B, H, W, D, 2.0)
    K = L * (2 * r + 1) ** 3
    w = prng.uniform(7304, (96, K), -K ** -0.5, K ** -0.5)
    b = prng.uniform(7305, (96,), -K ** -0.5, K ** -0.5)
    gy = prng.normal(7306, (B, 96, H, W, D))
    tw = torch.from_numpy(w.reshape(96, -1, 1, 1, 1)).to(DEV).requires_grad_(True)
    tb = torch.from_numpy(b).to(DEV).requires_grad_(True)
    blk = dvccorr.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV), L, r, precision="bf16")
    assert blk._grad_fmaps is None and blk._brick
    out = blk.lookup_convc1(torch.from_numpy(coords).to(DEV), tw, tb)
    (out * torch.from_numpy(gy).to(DEV)).sum().backward()
    mask = (out.detach().cpu().numpy() > 0).astype(np.float32)
    _pre, _r1, _r2, rw, rb = _oracle(f1, f2, coords, w, b, gy, mask, L, r, legacy)
    assert orc.rel_err(tw.grad.view(96, -1).cpu().numpy(), rw) <= TOL["bf16"]
    assert orc.rel_err(tb.grad.cpu().numpy(), rb) <= TOL["bf16"]


def test_lookup_convc1_ad_saves_no_lookup_tensor():
    """The autograd context of the fused op holds the (B, 96, Nq) output, not the (B, L*(2r+1)^3, Nq) lookup: peak
    memory of twelve forward iterations stays far below twelve lookup tensors (the unfused composition keeps one
    per iteration for conv3d's weight gradient)."""
    import dvccorr
    S, C, L, r = 16, 64, 4, 4
    g = torch.Generator(device=DEV).manual_seed(3)
    t1 = torch.randn(1, C, S, S, S, device=DEV, generator=g).requires_grad_(True)
    t2 = torch.randn(1, C, S, S, S, device=DEV, generator=g).requires_grad_(True)
    K = L * (2 * r + 1) ** 3
    tw = (torch.rand(96, K, 1, 1, 1, device=DEV, generator=g) * 2 - 1).mul_(K ** -0.5).requires_grad_(True)
    tb = torch.zeros(96, device=DEV, requires_grad=True)
    base = dvccorr.coords_grid_3d(1, S, S, S, DEV)
    blk = dvccorr.CorrBlock(t1, t2, L, r, precision="bf16")
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_allocated()
    outs = [blk.lookup_convc1(base + 0.5 * i, tw, tb) for i in range(12)]
    torch.cuda.synchronize()
    held = torch.cuda.memory_allocated() - m0
    lookup_bytes = K * S ** 3 * 4
    assert held < 2 * lookup_bytes, (held, lookup_bytes)   # twelve lookups would be 12 x lookup_bytes
    sum(o.sum() for o in outs).backward()
    assert t1.grad is not None and tw.grad is not None and torch.isfinite(t2.grad).all()
