#!/usr/bin/env python3
"""Generate the closed-loop flow fixture (north_star: <= 1e-3 voxel EPE on the final flow) -- survey
container only, by importing the reference.

    python tests/golden/gen_epe_golden.py [--reference /root/reference]

Config #1 (BASELINE): RAFTDVC, 64^3 volume pair, 1/8 encoder, L=4, r=4, 12 GRU iterations, test_mode.
The reference model is built with its seeded random init (as plumbing.npz), then its UPDATE BLOCK's
parameters are overwritten with values from the portable PRNG (tests/prng.py): uniform(-b, b), b =
1/sqrt(fan_in) of the owning Conv3d (PyTorch's default init range), one seed per parameter in
named_parameters() order.  The GPU harness (tests/raftdvc_loop.py) regenerates the same weights from
the seeds in epe_meta.json, so no weight tensor is stored.

Stored (epe_1_8.npz): the inputs of the refinement loop (raft_dvc.py:440-491) as the reference computed
them -- fmap0/fmap1 (CorrBlock's inputs, raft_dvc.py:366-367) and net/context (cnet output, :425) --
and its outputs: delta_flow of every iteration, the final low-res flow coords1 - coords0 (:495) and
checksums of flow_up.  Only reference OUTPUTS are written; no reference source is stored.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))

import prng  # noqa: E402

SEED_BASE = 7100


def checksums(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float64)
    return np.array([x.sum(), np.abs(x).sum(), (x * x).sum(), np.abs(x).max()], np.float64)


def update_block_params(block: torch.nn.Module):
    """[(name, shape, seed, bound)] for every parameter of the update block, in named_parameters() order."""
    fan = {}
    for mname, m in block.named_modules():
        if isinstance(m, torch.nn.Conv3d):
            w = m.weight
            fan[mname] = w.shape[1] * int(np.prod(w.shape[2:]))
    out = []
    for i, (name, p) in enumerate(block.named_parameters()):
        owner = name.rsplit(".", 1)[0]
        out.append((name, list(p.shape), SEED_BASE + i, 1.0 / float(np.sqrt(fan[owner]))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    sys.path.insert(0, a.reference)
    from src.core.raft_dvc import RAFTDVC, RAFTDVCConfig  # type: ignore
    torch.manual_seed(1234)
    cfg = RAFTDVCConfig(encoder_type="1/8", corr_levels=4, corr_radius=4, iters=12)
    model = RAFTDVC(cfg).eval()
    meta = update_block_params(model.update_block)
    with torch.no_grad():
        params = dict(model.update_block.named_parameters())
        for name, shape, seed, bound in meta:
            params[name].copy_(torch.from_numpy(prng.uniform(seed, tuple(shape), -bound, bound)))

    vol0 = torch.from_numpy(prng.uniform(301, (1, 1, 64, 64, 64)))
    vol1 = torch.roll(vol0, shifts=(2, -1, 3), dims=(2, 3, 4))
    cap = {"delta": [], "flow_in": []}
    ub = model.update_block
    orig_forward = ub.forward

    def spy(net, context, corr, flow):      # records the loop's inputs/outputs, behaviour unchanged
        if not cap["delta"]:
            cap["net0"] = net.detach().numpy().copy()
            cap["context"] = context.detach().numpy().copy()
        cap["flow_in"].append(flow.detach().numpy().copy())
        out = orig_forward(net, context, corr, flow)
        cap["delta"].append(out[1].detach().numpy().copy())
        return out

    import src.core.raft_dvc as rd  # type: ignore
    Orig = rd.CorrBlock

    class CorrSpy(Orig):
        def __init__(self, fmap1, fmap2, *args, **kw):
            cap["fmap0"] = fmap1.detach().numpy().copy()
            cap["fmap1"] = fmap2.detach().numpy().copy()
            super().__init__(fmap1, fmap2, *args, **kw)

    ub.forward = spy
    rd.CorrBlock = CorrSpy
    try:
        with torch.no_grad():
            flow_lo, flow_up = model(vol0, vol1, test_mode=True)
    finally:
        rd.CorrBlock = Orig
        ub.forward = orig_forward
    out = os.path.join(HERE, "epe_1_8.npz")
    np.savez_compressed(out, fmap0=cap["fmap0"], fmap1=cap["fmap1"], net0=cap["net0"], context=cap["context"],
                        delta=np.stack(cap["delta"]), flow_in=np.stack(cap["flow_in"]), flow_lo=flow_lo.numpy(),
                        flow_up_checksum=checksums(flow_up.numpy()), target_shape=np.array([64, 64, 64]))
    with open(os.path.join(HERE, "epe_meta.json"), "w") as f:
        json.dump({"torch": torch.__version__, "config": "RAFTDVC 1/8, L=4, r=4, hidden 96, context 64, sep-conv "
                   "GRU, 12 iters, test_mode; update-block weights uniform(-b, b) from tests/prng.py",
                   "params": meta, "flow_lo_absmax": float(np.abs(flow_lo.numpy()).max()),
                   "delta_absmax": [float(np.abs(d).max()) for d in cap["delta"]]}, f, indent=1)
    print("wrote", out, "flow_lo |max|", float(np.abs(flow_lo.numpy()).max()))


if __name__ == "__main__":
    main()
