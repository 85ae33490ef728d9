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
