#!/usr/bin/env python3
"""Golden vectors for the per-iteration flow ops -- survey container only.

    python tests/golden/gen_flow_golden.py [--reference /root/reference]

Imports the reference (zachtong/RAFT-DVC) from its read-only checkout and runs, on
CPU, its coords_grid_3d (src/core/corr.py:71-99), upflow_3d (corr.py:211-253) and
RAFTDVC.forward's coordinate update + upsampling (src/core/raft_dvc.py:482-485):

    coords1 = coords1 + delta_flow
    flow_up = upflow_3d(coords1 - coords0, target_shape=target_shape)

Inputs come from tests/prng.py streams (regenerated bit-identically anywhere);
only the outputs and the seeds/shapes are stored (flow_*.npz).
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

# name, B, (h, w, d) low-res, (H, W, D) target, max_flow, seed
CASES = [
    ("flow_8_to_64", 1, (8, 8, 8), (64, 64, 64), 3.0, 600),        # 1/8 encoder, cfg #1
    ("flow_978_to_x4", 2, (9, 7, 8), (36, 28, 32), 2.0, 610),       # non-cubic, 1/4 encoder
    ("flow_ceil_target", 1, (5, 6, 4), (17, 23, 15), 2.5, 620),     # ceil(H/8) grid, non-integer scales
    ("flow_size1_axis", 1, (4, 1, 3), (8, 5, 9), 1.5, 630),          # a size-1 source axis
]


def flow_inputs(B, lo, mf, seed):
    h, w, d = lo
    coords1 = prng.flow_coords(seed, B, h, w, d, mf)
    delta = prng.uniform(seed + 1, (B, 3, h, w, d), -1.0, 1.0)
    log_b = prng.uniform(seed + 2, (B, 3, h, w, d), -2.0, 2.0)
    return coords1, delta, log_b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    from src.core.corr import coords_grid_3d, upflow_3d  # type: ignore
    torch.set_num_threads(8)
    meta = {"torch": torch.__version__, "reference": "zachtong/RAFT-DVC @ /root/reference (read-only)",
            "fixtures": {}}
    for name, B, lo, tgt, mf, seed in CASES:
        c1, dl, lb = (torch.from_numpy(a) for a in flow_inputs(B, lo, mf, seed))
        coords0 = coords_grid_3d(B, *lo, device=torch.device("cpu"))
        coords1 = c1 + dl                                                   # raft_dvc.py:482
        flow_up = upflow_3d(coords1 - coords0, target_shape=tgt)            # raft_dvc.py:485
        log_b_up = upflow_3d(lb, target_shape=tgt)                          # raft_dvc.py:490
        up8 = upflow_3d(coords1 - coords0)                                  # scale_factor=8 branch
        # fixtures stay small: large outputs keep every hstep-th target plane (H axis),
        # the scale_factor=8 and log_b outputs only for the small cases
        small = up8.numel() < 300_000
        hstep = 1 if small else 3
        extra = {"log_b_up": log_b_up.numpy(), "up8": up8.numpy()} if small else {}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), coords0=coords0.numpy(), coords1=coords1.numpy(),
                            flow_up=flow_up[:, :, ::hstep].numpy(), hstep=np.array([hstep]),
                            shape=np.array([B, *lo, *tgt], np.int64), max_flow=np.array([mf]),
                            seed=np.array([seed]), **extra)
        meta["fixtures"][name] = {"flow_up": list(flow_up.shape), "up8": list(up8.shape)}
        print(f"  wrote {name}.npz flow_up {tuple(flow_up.shape)} max {float(flow_up.abs().max()):.3f}")
    with open(os.path.join(HERE, "flow_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
