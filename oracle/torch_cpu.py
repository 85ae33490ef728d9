"""torch-CPU restatement of the reference op sequence -- TEST/BASELINE ONLY.

This is the CPU column of the benchmark ("kind": "port"): the reference's
Python cannot travel to the GPU box, so bench.py times this restatement on
the box's host cores instead.  It runs the same op sequence as
zachtong/RAFT-DVC src/core/corr.py:
    matmul(fmap1^T, fmap2) / sqrt(C)             corr.py:155-167
    F.avg_pool3d(., 2, stride=2) per level       corr.py:136-139
    per level: centroid / 2**i + delta grid      corr.py:184-199
    normalise by (S-1), grid_sample trilinear,
    zeros, align_corners=True                    corr.py:41-63
    cat over levels, permute to (B, L*n^3, ...)  corr.py:207-208
and additionally supports a contiguous slab of query rows [q0, q1) so that
the 256^3 configurations (which do not fit host RAM) can be timed on a
bounded sample and extrapolated linearly (rows are independent).

tests/golden/gen_golden.py checks it bit-for-bit against the reference in
the survey container; tests/test_oracle_golden.py re-checks it against the
committed golden vectors.  Never imported by the product package.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def build_rows(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int, q0: int = 0, q1=None):
    """Correlation pyramid for query rows [q0, q1) of every batch element.

    Returns a list of num_levels tensors shaped (B*(q1-q0), 1, H_l, W_l, D_l).
    """
    B, C, H, W, D = fmap1.shape
    N = H * W * D
    q1 = N if q1 is None else q1
    lhs = fmap1.reshape(B, C, N)[:, :, q0:q1].transpose(1, 2)
    cost = torch.matmul(lhs, fmap2.reshape(B, C, N))
    cost = cost / torch.sqrt(torch.tensor(C, dtype=torch.float32, device=cost.device))
    level = cost.reshape(B * (q1 - q0), 1, H, W, D)
    pyramid = [level]
    for _ in range(num_levels - 1):
        level = F.avg_pool3d(level, 2, stride=2)
        pyramid.append(level)
    return pyramid


def _sample(vol: torch.Tensor, pts: torch.Tensor, legacy: bool) -> torch.Tensor:
    """vol (M, 1, S_h, S_w, S_d); pts (M, n, n, n, 3) in (h, w, d) order."""
    _, _, Sh, Sw, Sd = vol.shape
    g = pts.clone()
    g[..., 0] = 2.0 * g[..., 0] / (Sh - 1) - 1.0
    g[..., 1] = 2.0 * g[..., 1] / (Sw - 1) - 1.0
    g[..., 2] = 2.0 * g[..., 2] / (Sd - 1) - 1.0
    order = [2, 0, 1] if legacy else [1, 0, 2]
    g = g[..., order].permute(0, 3, 1, 2, 4)
    res = F.grid_sample(vol.permute(0, 1, 4, 2, 3), g, mode="bilinear", padding_mode="zeros",
                        align_corners=True)
    return res.permute(0, 1, 3, 4, 2)


def lookup_rows(pyramid, coords: torch.Tensor, radius: int, legacy: bool = False,
                q0: int = 0, q1=None) -> torch.Tensor:
    """Lookup for query rows [q0, q1): coords (B, 3, H, W, D) -> (B, L*n^3, q1-q0)."""
    B = coords.shape[0]
    N = coords[0, 0].numel()
    q1 = N if q1 is None else q1
    nq = q1 - q0
    cr = coords.reshape(B, 3, N)[:, :, q0:q1].permute(0, 2, 1).reshape(B * nq, 1, 1, 1, 3)
    n = 2 * radius + 1
    steps = torch.linspace(-radius, radius, n, device=coords.device)
    offs = torch.stack(torch.meshgrid(steps, steps, steps, indexing="ij"), dim=-1).reshape(1, n, n, n, 3)
    outs = []
    for i, vol in enumerate(pyramid):
        pts = cr / 2 ** i + offs
        outs.append(_sample(vol, pts, legacy).reshape(B, nq, -1))
    return torch.cat(outs, dim=-1).permute(0, 2, 1).contiguous().float()


def corr_lookup(fmap1, fmap2, coords, num_levels=4, radius=4, legacy=False):
    """Full build + one lookup -> (B, L*n^3, H, W, D) float32."""
    B, C, H, W, D = fmap1.shape
    pyr = build_rows(fmap1, fmap2, num_levels)
    return lookup_rows(pyr, coords, radius, legacy).reshape(B, -1, H, W, D)
