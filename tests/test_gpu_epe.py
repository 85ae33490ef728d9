"""Closed-loop parity on the final flow (north_star: <= 1e-3 voxel EPE), config #1.

RAFTDVC 64^3, 1/8 encoder, L=4, r=4, 12 GRU iterations: the reference's own refinement loop
(raft_dvc.py:440-491) is run with dvccorr in place of CorrBlock (corr.py:116-208) and of the iteration
tail (raft_dvc.py:482-485: dvccorr.flow_step), the update block (update.py) restated in torch on the GPU
(tests/raftdvc_loop.py, pinned on CPU by test_epe_cpu.py).  The loop starts from the reference's fmaps and
cnet outputs (tests/golden/epe_1_8.npz) and its final low-res flow is compared with the reference's:
ulp-level differences in the lookup pass through 12 nonlinear GRU updates, so this is where they would
amplify.  A same-GPU torch path (reference op sequence on the GPU) measures the floor that the
GPU's own conv/grid_sample arithmetic sets.
"""
from __future__ import annotations

import pytest
import torch

import raftdvc_loop as rl
from conftest import load_golden
from oracle import torch_cpu

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
EPE_TOL = 1e-3


def _run(kind):
    import dvccorr
    g = load_golden("epe_1_8.npz")
    p = rl.load_params(DEV)
    f0, f1 = torch.from_numpy(g["fmap0"]).to(DEV), torch.from_numpy(g["fmap1"]).to(DEV)
    B, _, h, w, d = f0.shape
    coords0 = dvccorr.coords_grid_3d(B, h, w, d, DEV)
    T = tuple(int(v) for v in g["target_shape"])
    net, ctx = torch.from_numpy(g["net0"]).to(DEV), torch.from_numpy(g["context"]).to(DEV)
    tail = lambda c, dl: dvccorr.flow_step(c, dl, T)          # noqa: E731
    convc1 = False
    if kind == "torch_gpu":      # the reference op sequence on the GPU: the floor of GPU arithmetic
        lookup = lambda c: torch_cpu.corr_lookup(f0, f1, c, 4, 4, False)     # noqa: E731
        tail = lambda c, dl: rl.reference_tail(c, dl, coords0, T)           # noqa: E731
    elif kind in ("fp32", "bf16", "fp16"):
        lookup = dvccorr.CorrBlock(f0, f1, 4, 4, precision=kind)
    elif kind in ("fused_fp32", "fused_bf16", "fused_fp16"):
        lookup = dvccorr.CorrBlockFused(f0, f1, 4, 4, precision=kind.split("_")[1])
    elif kind in ("bf16_convc1", "fp16_convc1", "fused_fp16_convc1"):
        prec = "fp16" if "fp16" in kind else "bf16"
        cls = dvccorr.CorrBlockFused if kind.startswith("fused") else dvccorr.CorrBlock
        blk = cls(f0, f1, 4, 4, precision=prec)
        lookup = lambda c: blk.lookup_convc1(c, p["encoder.convc1.weight"], p["encoder.convc1.bias"])  # noqa
        convc1 = True
    with torch.no_grad():
        flow_lo, flow_up, _ = rl.refine(lookup, tail, p, net, ctx, coords0, 12, T, convc1=convc1)
    torch.cuda.synchronize()
    return rl.epe(flow_lo, g["flow_lo"]), flow_up


# fp16 (round 4): the reference Trainer's AMP precision on both blocks and the fused convc1 paths
@pytest.mark.parametrize("kind", ["torch_gpu", "fp32", "fused_fp32", "bf16", "fused_bf16", "bf16_convc1", "fp16",
                                  "fused_fp16", "fp16_convc1", "fused_fp16_convc1"])
def test_final_flow_epe(kind):
    e, flow_up = _run(kind)
    print(f"EPE[{kind}] = {e:.3e} voxel")
    assert torch.isfinite(flow_up).all()
    assert e <= EPE_TOL, (kind, e)
