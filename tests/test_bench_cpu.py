"""CPU checks of bench.py's host logic: the --gpus N spawn path (a parent that never touches the GPU
launches torch.distributed.run with N ranks on 127.0.0.1) and the algorithmic-byte model of SURVEY 8(d)."""
from __future__ import annotations

import os
import sys

import pytest
import torch

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_gpus_flag_spawns_torchrun(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a: pytest.fail("the parent touched the GPU"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7                      # exits with the child's code
    (cmd,) = calls
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.abspath(bench.__file__)) + 1:] == ["--gpus", "4", "--steps", "2"]


def test_world_size_must_match(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()


def test_defaults_are_strong_scaling_graph_replay():
    a = bench.parse([])
    assert a.scaling == "strong" and a.graph and a.gpus == 1 and a.size == 32 and a.levels == 4


def test_lookup_algorithmic_bytes_brute_force():
    """|W_l(q)| = touched integer window clipped to the level, brute-forced on a small grid."""
    g = torch.Generator().manual_seed(0)
    H, W, D, r = 6, 5, 7, 2
    dims = [(H, W, D), (3, 2, 3)]
    coords = torch.rand(1, 3, H * W * D, generator=g) * torch.tensor([H, W, D]).view(1, 3, 1) * 1.4 - 1.0
    got = bench.lookup_algorithmic_bytes(coords, dims, r, 2)
    win = 0
    for q in range(H * W * D):
        for l, (h, w, d) in enumerate(dims):
            n = 1
            for ax, s in enumerate((h, w, d)):
                k = int(torch.floor(coords[0, ax, q] / 2 ** l))
                n *= sum(1 for i in range(k - r, k + r + 2) if 0 <= i < s)
            win += n
    n3 = (2 * r + 1) ** 3
    assert got == pytest.approx(win * 2 + H * W * D * (4 * 2 * n3 + 12))


@pytest.mark.parametrize("kind", ["random", "smooth"])
def test_synthetic_flow_bounded_and_seeded(kind):
    """--flow random (the default: i.i.d. per voxel and axis) and --flow smooth (three sinusoids per axis) stay
    within +-max_flow and are reproducible from the generator seed; the smooth field varies slowly."""
    g1, g2 = torch.Generator().manual_seed(11), torch.Generator().manual_seed(11)
    a = bench.synthetic_flow(kind, 2, 16, 2.0, g1)
    b = bench.synthetic_flow(kind, 2, 16, 2.0, g2)
    assert a.shape == (2, 3, 16, 16, 16) and torch.equal(a, b)
    assert float(a.abs().max()) <= 2.0 + 1e-6
    step = max(float((a.diff(dim=d)).abs().max()) for d in (2, 3, 4))
    if kind == "smooth":
        assert step < 2.0 * 2 * torch.pi * 2 / 16   # |d/dp| <= 3 * (2/3) * 2 pi |k| / S per voxel
    else:
        assert step > 2.0                           # i.i.d.: neighbours differ by up to 4
