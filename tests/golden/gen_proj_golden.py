#!/usr/bin/env python3
"""Golden vectors for the convc1-fused lookup -- survey container only.

    python tests/golden/gen_proj_golden.py [--reference /root/reference]

Imports the reference (zachtong/RAFT-DVC) from its read-only checkout and runs,
on CPU, its CorrBlock (src/core/corr.py:116-208) followed by its MotionEncoder's
first layer, F.relu(self.convc1(corr)) (src/core/update.py:219-222, 246), with
convc1's weight and bias set from tests/prng.py streams.  Only the OUTPUTS and
the seeds/shapes are stored (proj_*.npz); tests/prng.py regenerates the inputs
bit-identically anywhere.
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

# name, B, C, (H, W, D), L, r, legacy, max_flow, seed
CASES = [
    ("proj_888_L2_r4", 1, 16, (8, 8, 8), 2, 4, False, 2.0, 500),
    ("proj_888_L2_r4_legacy", 1, 16, (8, 8, 8), 2, 4, True, 2.0, 510),
    ("proj_978_L3_r3", 1, 16, (9, 7, 8), 3, 3, False, 2.5, 520),
    ("proj_888_L2_r2_legacy", 2, 16, (8, 8, 8), 2, 2, True, 1.5, 530),
    ("proj_888_L4_r1", 1, 32, (8, 8, 8), 4, 1, False, 3.0, 540),
]


def proj_inputs(B, C, shape, L, r, max_flow, seed):
    """fmaps, coords, convc1 weight (96, L (2r+1)^3) and bias, PyTorch's default Conv3d init range."""
    H, W, D = shape
    f1 = prng.normal(seed, (B, C, H, W, D))
    f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, max_flow)
    K = L * (2 * r + 1) ** 3
    bound = 1.0 / np.sqrt(K)
    w = prng.uniform(seed + 3, (96, K), -bound, bound)
    b = prng.uniform(seed + 4, (96,), -bound, bound)
    return f1, f2, coords, w, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    from src.core.corr import CorrBlock  # type: ignore
    from src.core.update import MotionEncoder  # type: ignore
    torch.set_num_threads(8)
    meta = {"torch": torch.__version__, "reference": "zachtong/RAFT-DVC @ /root/reference (read-only)",
            "fixtures": {}}
    for name, B, C, shape, L, r, legacy, mf, seed in CASES:
        f1, f2, coords, w, b = proj_inputs(B, C, shape, L, r, mf, seed)
        enc = MotionEncoder(corr_levels=L, corr_radius=r)
        with torch.no_grad():
            enc.convc1.weight.copy_(torch.from_numpy(w).view(96, -1, 1, 1, 1))
            enc.convc1.bias.copy_(torch.from_numpy(b))
            blk = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r,
                            legacy_wd_swap=legacy)
            corr = blk(torch.from_numpy(coords))
            out = torch.relu(enc.convc1(corr))     # update.py:246
        np.savez_compressed(os.path.join(HERE, name + ".npz"), out=out.numpy().astype(np.float32),
                            shape=np.array([B, C, *shape, L, r], np.int64), legacy=np.array([int(legacy)]),
                            max_flow=np.array([mf]), seed=np.array([seed]))
        meta["fixtures"][name] = list(out.shape)
        print(f"  wrote {name}.npz {tuple(out.shape)} max {float(out.abs().max()):.3f}")
    with open(os.path.join(HERE, "proj_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
