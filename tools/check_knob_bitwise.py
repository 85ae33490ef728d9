#!/usr/bin/env python3
"""Bitwise comparison of the config #3 lookup (bricked bf16 pyramid, the product path) under two knob sets.
    python tools/check_knob_bitwise.py "lookup_lmix=0" "lookup_lmix=1" [--size 32]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))
import dvccorr  # noqa: E402
from dvccorr import _lib  # noqa: E402

a, b = sys.argv[1], sys.argv[2]
S = int(sys.argv[sys.argv.index("--size") + 1]) if "--size" in sys.argv else 32
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(7)
f1 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
f2 = torch.randn(1, 128, S, S, S, generator=g).to(dev)
base = torch.stack(torch.meshgrid(*[torch.arange(S, dtype=torch.float32)] * 3, indexing="ij"))[None]
c = (base + (torch.rand(1, 3, S, S, S, generator=g) * 4 - 2)).to(dev)
c[0, :, 0, 0, :3] = float("nan")
with torch.no_grad():
    outs = []
    for ks in (a, b):   # (the knobs are set before the block packs and builds its pyramid)
        for item in filter(None, ks.split(",")):
            k, v = item.split("=")
            _lib.set_tuning(k, int(v))
        blk = dvccorr.CorrBlock(f1, f2, 4, 4, precision="bf16")
        outs.append(blk(c).clone())
        del blk
        torch.cuda.synchronize()
eq = torch.equal(torch.nan_to_num(outs[0], nan=7.0), torch.nan_to_num(outs[1], nan=7.0))
print("bitwise equal:", eq, "max diff", (outs[0] - outs[1]).abs().nan_to_num(0).max().item())
sys.exit(0 if eq else 1)
