"""pytest setup: markers, import paths, fixture helpers.

`-m gpu` tests need an MI355X (the HIP library is the thing under test);
`-m "not gpu"` tests run on CPU: the oracle against the golden vectors, host
logic, layout helpers, the C-ABI library's exported symbols and the
multi-rank (gloo) sharding logic.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "raft-dvc_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP library under test)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name: str):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    return load_golden


def corr_inputs(g):
    """Regenerate a corr_case fixture's inputs from its seeds (tests/prng.py)."""
    import prng
    B, C, H, W, D, L, r = (int(v) for v in g["shape"])
    s = [int(v) for v in g["seeds"]]
    f1 = prng.normal(s[0], (B, C, H, W, D))
    f2 = prng.normal(s[1], (B, C, H, W, D))
    coords = prng.flow_coords(s[2], B, H, W, D, float(g["max_flow"][0]))
    return f1, f2, coords, L, r


def grad_inputs(g):
    """Regenerate a grad_* fixture's inputs (tests/golden/gen_grad_golden.py): fmaps, coords, the output
    gradient G (all ones or N(0,1)), L, r, legacy."""
    import prng
    B, C, H, W, D, L, r = (int(v) for v in g["shape"])
    s = [int(v) for v in g["seeds"]]
    f1 = prng.normal(s[0], (B, C, H, W, D))
    f2 = prng.normal(s[1], (B, C, H, W, D))
    coords = prng.flow_coords(s[2], B, H, W, D, float(g["max_flow"][0]))
    gshape = (B, L * (2 * r + 1) ** 3, H, W, D)
    G = np.ones(gshape, np.float32) if int(g["gkind"][0]) == 0 else prng.normal(s[3], gshape)
    return f1, f2, coords, G, L, r, bool(int(g["legacy"][0]))


def oracle_grads(f1, f2, coords, G, L, r, legacy):
    """The backward oracle: autograd through oracle/torch_cpu.py (bit-identical to the reference's autograd on
    every grad_* fixture, tests/golden/grad_meta.json)."""
    import torch
    from oracle import torch_cpu
    t1 = torch.from_numpy(np.ascontiguousarray(f1)).requires_grad_(True)
    t2 = torch.from_numpy(np.ascontiguousarray(f2)).requires_grad_(True)
    out = torch_cpu.corr_lookup(t1, t2, torch.from_numpy(np.ascontiguousarray(coords)), L, r, legacy)
    (out * torch.from_numpy(np.ascontiguousarray(G))).sum().backward()
    return t1.grad.numpy(), t2.grad.numpy()


def proj_inputs(g):
    """Regenerate a proj_* fixture's inputs (tests/golden/gen_proj_golden.py): fmaps, coords, convc1 weight
    (96, L (2r+1)^3) and bias, L, r, legacy."""
    import prng
    B, C, H, W, D, L, r = (int(v) for v in g["shape"])
    seed = int(g["seed"][0])
    f1 = prng.normal(seed, (B, C, H, W, D))
    f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, float(g["max_flow"][0]))
    K = L * (2 * r + 1) ** 3
    bound = 1.0 / np.sqrt(K)
    w = prng.uniform(seed + 3, (96, K), -bound, bound)
    b = prng.uniform(seed + 4, (96,), -bound, bound)
    return f1, f2, coords, w, b, L, r, bool(g["legacy"][0])
