#!/usr/bin/env python3
"""Golden vectors for the AMP (fp16) pyramid -- survey container only.

    python tests/golden/gen_amp_golden.py [--reference /root/reference]

The reference Trainer runs RAFTDVC.forward under torch.amp.autocast('cuda')
(src/training/trainer.py:249-252), so CorrBlock's torch.matmul (corr.py:161)
runs in float16 and the whole pyramid is float16 (corr.py:155-167), while the
lookup output is cast back to float32 (corr.py:208).  There is no CUDA device
here, so the reference CorrBlock is run on CPU under
torch.autocast('cpu', dtype=torch.float16): the matmul and the divide by
sqrt(C) run in float16 exactly as on CUDA; CPU autocast runs avg_pool3d in
float32 (CUDA runs it in float16 on the float16 level), so levels >= 1 here
are the float32 pools of the float16 level 0 -- within one float16 rounding of
the CUDA pyramid.  grid_sample runs in float32 on both (autocast fp32 list /
the .float() cast).

Inputs come from tests/prng.py (regenerated bit-identically anywhere); only
the OUTPUTS, seeds and shapes are stored (amp_*.npz).  Nothing from the
reference's source is stored.
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
    ("amp_888_L2_r4", 2, 16, (8, 8, 8), 2, 4, False, 2.0, 700),
    ("amp_888_L4_r4", 1, 32, (8, 8, 8), 4, 4, False, 2.0, 710),       # level 3 is 1^3: zeros
    ("amp_978_L3_r3", 1, 64, (9, 7, 8), 3, 3, False, 2.5, 720),
    ("amp_888_L3_r3_legacy", 1, 16, (8, 8, 8), 3, 3, True, 2.0, 730),
    ("amp_16_L4_r4_c128", 1, 128, (16, 16, 16), 4, 4, False, 2.0, 740),   # config #2's fmap shape
]


def amp_inputs(B, C, shape, max_flow, seed):
    H, W, D = shape
    f1 = prng.normal(seed, (B, C, H, W, D))
    f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, max_flow)
    return f1, f2, coords


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    from src.core.corr import CorrBlock  # type: ignore
    torch.set_num_threads(8)
    meta = {"torch": torch.__version__, "reference": "zachtong/RAFT-DVC @ /root/reference (read-only)",
            "autocast": "torch.autocast('cpu', dtype=torch.float16): matmul + /sqrt(C) in float16, "
                        "avg_pool3d in float32 on the float16 level 0 (CUDA pools in float16), grid_sample float32",
            "fixtures": {}}
    for name, B, C, shape, L, r, legacy, mf, seed in CASES:
        f1, f2, coords = amp_inputs(B, C, shape, mf, seed)
        with torch.no_grad(), torch.autocast("cpu", dtype=torch.float16):
            blk = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r,
                            legacy_wd_swap=legacy)
            dtypes = [str(p.dtype) for p in blk.corr_pyramid]
            out = blk(torch.from_numpy(coords))
        with torch.no_grad():   # the same call in float32, to record how far AMP moves the output
            ref32 = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r,
                              legacy_wd_swap=legacy)(torch.from_numpy(coords))
        assert out.dtype == torch.float32, out.dtype
        o = out.numpy().astype(np.float32)
        d32 = float(np.abs(o - ref32.numpy()).max() / max(np.abs(ref32.numpy()).max(), 1e-30))
        extra = {"out": o}
        if o.size > 4_000_000:   # large case: 256 sampled query rows (global row b*N + q) of every channel
            N = int(np.prod(shape))
            rows = np.unique((prng.uniform24(seed + 9, 1024) * (B * N)).astype(np.int64))[:256]
            flat = o.reshape(B, o.shape[1], N)
            extra = {"rows": rows, "out_rows": np.stack([flat[q // N, :, q % N] for q in rows]).astype(np.float32)}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **extra,
                            shape=np.array([B, C, *shape, L, r], np.int64), legacy=np.array([int(legacy)]),
                            max_flow=np.array([mf]), seed=np.array([seed]))
        meta["fixtures"][name] = {"out": list(o.shape), "pyramid_dtypes": dtypes, "rel_diff_vs_fp32": d32}
        print(f"  wrote {name}.npz {tuple(o.shape)} pyramid {dtypes} AMP vs fp32 {d32:.2e}")
    with open(os.path.join(HERE, "amp_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
