"""Test-only harness: RAFT-DVC's update block and refinement loop, restated functionally in torch, for the
closed-loop final-flow check (north_star: <= 1e-3 voxel EPE).  TEST INFRASTRUCTURE, never product code.

Restates the reference's math (zachtong/RAFT-DVC):
  MotionEncoder.forward        src/core/update.py:231-253   relu(convc1), relu(convf1/convf2), relu(conv), cat flow
  SepConvGRU3D.forward         src/core/update.py:167-199   h, w, d passes of the z / r / q gates
  FlowHead.forward             src/core/update.py:30-38     conv2(relu(conv1(h)))
  BasicUpdateBlock.forward     src/core/update.py:316-348   cat(context, motion) -> GRU -> flow head
  refinement loop              src/core/raft_dvc.py:440-491 corr = corr_fn(coords1); flow = coords1 - coords0;
                                                            update; coords1 += delta; flow_up = upflow_3d(...)
The parameters are the update block's named_parameters() regenerated from the portable PRNG with the seeds
and ranges tests/golden/gen_epe_golden.py wrote to epe_meta.json (the reference ran with the same values).
The correlation block and the iteration tail are pluggable: the reference-equivalent CPU restatement
(oracle/torch_cpu.py + F.interpolate) pins this harness against the fixture, dvccorr's HIP blocks and
flow_step are what the GPU test closes the loop on.
"""
from __future__ import annotations

import json
import os

import torch
import torch.nn.functional as F

import prng

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_params(device, meta_path=os.path.join(GOLDEN, "epe_meta.json")):
    with open(meta_path) as f:
        meta = json.load(f)
    return {name: torch.from_numpy(prng.uniform(seed, tuple(shape), -b, b)).to(device)
            for name, shape, seed, b in meta["params"]}


def _conv(p, name, x, padding):
    return F.conv3d(x, p[name + ".weight"], p[name + ".bias"], padding=padding)


def motion_features(p, flow, corr=None, cor=None):
    """update.py:246-253; `cor` = relu(convc1(corr)) when the lookup already applied convc1."""
    if cor is None:
        cor = F.relu(_conv(p, "encoder.convc1", corr, 0))
    flo = F.relu(_conv(p, "encoder.convf1", flow, 3))
    flo = F.relu(_conv(p, "encoder.convf2", flo, 1))
    out = F.relu(_conv(p, "encoder.conv", torch.cat([cor, flo], dim=1), 1))
    return torch.cat([out, flow], dim=1)


def sep_gru(p, h, x):
    """update.py:178-199: one z / r / q gate triple per axis, kernel 5 along that axis."""
    for ax, pad in (("h", (2, 0, 0)), ("w", (0, 2, 0)), ("d", (0, 0, 2))):
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(_conv(p, f"gru.convz_{ax}", hx, pad))
        r = torch.sigmoid(_conv(p, f"gru.convr_{ax}", hx, pad))
        q = torch.tanh(_conv(p, f"gru.convq_{ax}", torch.cat([r * h, x], dim=1), pad))
        h = (1 - z) * h + z * q
    return h


def update_block(p, net, context, flow, corr=None, cor=None):
    """update.py:338-342 (uncertainty_mode 'none')."""
    inp = torch.cat([context, motion_features(p, flow, corr, cor)], dim=1)
    net = sep_gru(p, net, inp)
    delta = _conv(p, "flow_head.conv2", F.relu(_conv(p, "flow_head.conv1", net, 1)), 1)
    return net, delta


def reference_tail(coords1, delta, coords0, target_shape):
    """raft_dvc.py:482-485 with corr.py:211-253 (the reference's own ops)."""
    coords1 = coords1 + delta
    flow = coords1 - coords0
    up = F.interpolate(flow, size=tuple(target_shape), mode="trilinear", align_corners=True)
    for c in range(3):
        up[:, c] *= target_shape[c] / flow.shape[2 + c]
    return coords1, up


def refine(lookup, tail, p, net, context, coords0, iters=12, target_shape=(64, 64, 64), convc1=False):
    """raft_dvc.py:440-491.  lookup(coords1) -> corr (or cor when convc1=True); tail(coords1, delta) ->
    (coords1, flow_up).  Returns (flow_lo, flow_up, per-iteration deltas)."""
    coords1 = coords0.clone()
    deltas = []
    flow_up = None
    for _ in range(iters):
        feat = lookup(coords1)
        flow = coords1 - coords0
        if convc1:
            net, delta = update_block(p, net, context, flow, cor=feat)
        else:
            net, delta = update_block(p, net, context, flow, corr=feat)
        deltas.append(delta)
        coords1, flow_up = tail(coords1, delta)
    return coords1 - coords0, flow_up, deltas


def epe(flow, ref) -> float:
    """Mean end-point error in voxels: mean over voxels of the L2 norm of the 3-vector difference."""
    d = (torch.as_tensor(flow).double().cpu() - torch.as_tensor(ref).double().cpu())
    return float(d.pow(2).sum(dim=1).sqrt().mean())
