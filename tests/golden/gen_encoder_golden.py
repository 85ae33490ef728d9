#!/usr/bin/env python3
"""Golden outputs of the reference feature encoders for the sharded-encoder tests -- survey container only.

    python tests/golden/gen_encoder_golden.py [--reference /root/reference]

BasicEncoder (1/8), MediumEncoder (1/4), ShallowEncoder (1/2) of zachtong/RAFT-DVC src/core/extractor.py
with instance norm, their parameters set from the portable PRNG (tests/raftdvc_encoder.set_params, the
same seeds and order), run in eval mode on a seeded input volume.  Only the outputs are stored
(encoder_*.npz); tests/raftdvc_encoder.py restates the architecture and must reproduce them.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import prng  # noqa: E402
import raftdvc_encoder as renc  # noqa: E402

CASES = {"1_8": ("1/8", "BasicEncoder", (32, 24, 16)), "1_4": ("1/4", "MediumEncoder", (32, 24, 16)),
         "1_2": ("1/2", "ShallowEncoder", (16, 12, 8))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    sys.path.insert(0, a.reference)
    from src.core import extractor  # type: ignore
    for tag, (kind, cls, shape) in CASES.items():
        ref = getattr(extractor, cls)(input_dim=1, output_dim=128, norm_fn="instance").eval()
        mine = renc.Encoder(kind).eval()
        names_r = [n for n, _ in ref.named_parameters()]
        names_m = [n for n, _ in mine.named_parameters()]
        assert names_r == names_m, (tag, set(names_r) ^ set(names_m))
        seed0 = 8000 + 100 * len(tag) + ord(tag[-1])
        renc.set_params(ref, seed0)
        renc.set_params(mine, seed0)
        x = torch.from_numpy(prng.uniform(8500 + ord(tag[-1]), (1, 1) + shape))
        with torch.no_grad():
            out = ref(x)
            err = float((mine(x) - out).abs().max() / out.abs().max())
        print(tag, cls, tuple(out.shape), "restatement rel err", err)
        np.savez_compressed(os.path.join(HERE, f"encoder_{tag}.npz"), out=out.numpy(), seed0=np.array([seed0]),
                            in_seed=np.array([8500 + ord(tag[-1])]), in_shape=np.array((1, 1) + shape),
                            restatement_err=np.array([err]))


if __name__ == "__main__":
    main()
