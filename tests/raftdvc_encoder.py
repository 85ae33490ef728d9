"""Test-only restatement of RAFT-DVC's feature encoders (TEST INFRASTRUCTURE, never product code).

zachtong/RAFT-DVC src/core/extractor.py:
  BottleneckBlock3D   :72-141   1x1 -> 3x3 (stride s) -> 1x1 convs with norms, ReLU, 1x1-stride-s shortcut
  BasicEncoder (1/8)  :142-256  conv1 7^3/2 + norm + ReLU, layers 32/1, 64/2, 96/2, conv2 1x1 -> output_dim
  MediumEncoder (1/4) :304-412  layers 32/1, 64/2, 96/1
  ShallowEncoder(1/2) :415-523  layers 32/1, 64/1, 96/1
with the reference's attribute names, so a state dict or the sharded encoder
(dvccorr.sharded_encoder) sees the same module tree.  Pinned against the reference by
tests/golden/encoder_*.npz (gen_encoder_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import prng

STRIDES = {"1/8": (1, 2, 2), "1/4": (1, 2, 1), "1/2": (1, 1, 1)}


class Bottleneck(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        mid = cout // 4
        self.conv1 = nn.Conv3d(cin, mid, 1)
        self.conv2 = nn.Conv3d(mid, mid, 3, padding=1, stride=stride)
        self.conv3 = nn.Conv3d(mid, cout, 1)
        self.norm1, self.norm2, self.norm3 = nn.InstanceNorm3d(mid), nn.InstanceNorm3d(mid), nn.InstanceNorm3d(cout)
        self.relu = nn.ReLU()
        self.downsample = None
        if stride != 1 or cin != cout:
            self.norm4 = nn.InstanceNorm3d(cout)
            self.downsample = nn.Sequential(nn.Conv3d(cin, cout, 1, stride=stride), self.norm4)

    def forward(self, x):
        y = F.relu(self.norm1(self.conv1(x)))
        y = F.relu(self.norm2(self.conv2(y)))
        y = self.norm3(self.conv3(y))
        return F.relu(y + (x if self.downsample is None else self.downsample(x)))


class Encoder(nn.Module):
    # forward is extractor.py's conv1 -> norm1 -> relu -> layers -> conv2 (the sequence ShardedEncoder interprets)
    sharded_forward_equivalent = True

    def __init__(self, kind="1/4", input_dim=1, output_dim=128):
        super().__init__()
        s1, s2, s3 = STRIDES[kind]
        self.conv1 = nn.Conv3d(input_dim, 32, 7, stride=2, padding=3)
        self.norm1 = nn.InstanceNorm3d(32)
        self.relu1 = nn.ReLU()
        self.layer1 = nn.Sequential(Bottleneck(32, 32, s1), Bottleneck(32, 32, 1))
        self.layer2 = nn.Sequential(Bottleneck(32, 64, s2), Bottleneck(64, 64, 1))
        self.layer3 = nn.Sequential(Bottleneck(64, 96, s3), Bottleneck(96, 96, 1))
        self.conv2 = nn.Conv3d(96, output_dim, 1)
        self.dropout = None

    def forward(self, x):
        x = F.relu(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        return self.conv2(x)


def set_params(module: nn.Module, seed0: int) -> None:
    """Every parameter (named_parameters order) <- uniform(-b, b) from the portable PRNG, b = 1/sqrt(fan_in)
    of its Conv3d (the generator applies the same values to the reference module)."""
    fan = {n: m.weight.shape[1] * int(torch.tensor(m.weight.shape[2:]).prod())
           for n, m in module.named_modules() if isinstance(m, nn.Conv3d)}
    with torch.no_grad():
        for i, (name, p) in enumerate(module.named_parameters()):
            b = fan[name.rsplit(".", 1)[0]] ** -0.5
            p.copy_(torch.from_numpy(prng.uniform(seed0 + i, tuple(p.shape), -b, b)))
