"""CPU, multi-process (gloo): query-voxel sharding of the correlation block.

The per-rank compute is swapped for the torch-CPU restatement of the
reference (oracle/torch_cpu.py) through ShardedCorrBlock's backend hook, so
what is under test is the partitioning, the fmap2 all-gather and the output
gather -- the same code the RCCL run on the GPUs executes.  World sizes 2 and
3 (uneven slabs), both conventions.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


class TorchCpuRows:
    """Backend: this rank's rows [q_offset, q_offset + Nq) via the reference op sequence."""

    def __init__(self, q_flat, fmap2, num_levels, radius, legacy, precision, impl, q_offset=0):
        from oracle import torch_cpu
        self.tc = torch_cpu
        B, C, Nq = q_flat.shape
        _, _, H, W, D = fmap2.shape
        self.dims = (B, H, W, D)
        self.q0, self.q1 = q_offset, q_offset + Nq
        f1 = torch.zeros(B, C, H * W * D)
        f1[:, :, self.q0:self.q1] = q_flat
        self.pyr = torch_cpu.build_rows(f1.view(B, C, H, W, D), fmap2, num_levels, self.q0, self.q1)
        self.R, self.legacy = radius, legacy

    def lookup(self, coords_flat):
        B, H, W, D = self.dims
        c = torch.zeros(B, 3, H * W * D)
        c[:, :, self.q0:self.q1] = coords_flat
        return self.tc.lookup_rows(self.pyr, c.view(B, 3, H, W, D), self.R, self.legacy, self.q0, self.q1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shape, L, R, q):
    import sys
    for p in (REPO, PKG, os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import prng
        from dvccorr.sharded import ShardedCorrBlock, slab_bounds
        B, C, H, W, D = shape
        f1 = torch.from_numpy(prng.normal(41, shape))
        f2 = torch.from_numpy(prng.normal(42, shape))
        coords = torch.from_numpy(prng.flow_coords(43, B, H, W, D, 2.0))
        h0, h1 = slab_bounds(H, world, rank)
        res = {}
        for legacy in (False, True):
            blk = ShardedCorrBlock(f1[:, :, h0:h1].contiguous(), f2[:, :, h0:h1].contiguous(), H, L, R, legacy,
                                   precision="fp32", backend=TorchCpuRows, gather_output=True)
            full = blk(coords[:, :, h0:h1].contiguous())
            blk.gather_output = False
            local = blk(coords[:, :, h0:h1].contiguous())
            res[legacy] = (full.numpy(), local.numpy(), (h0, h1))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape", [(2, (1, 16, 8, 8, 8)), (3, (2, 8, 9, 7, 8))])
def test_sharded_matches_single_process(world, shape):
    from oracle import torch_cpu
    import prng
    L, R = (2, 3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, L, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B, C, H, W, D = shape
    f1 = torch.from_numpy(prng.normal(41, shape))
    f2 = torch.from_numpy(prng.normal(42, shape))
    coords = torch.from_numpy(prng.flow_coords(43, B, H, W, D, 2.0))
    for legacy in (False, True):
        ref = torch_cpu.corr_lookup(f1, f2, coords, L, R, legacy).numpy()
        for r in range(world):
            full, local, (h0, h1) = results[r][legacy]
            assert full.shape == ref.shape
            np.testing.assert_allclose(full, ref, rtol=0, atol=2e-6 * np.abs(ref).max())
            np.testing.assert_allclose(local, ref[:, :, h0:h1], rtol=0, atol=2e-6 * np.abs(ref).max())
        # every rank's gathered output is identical (same bytes everywhere)
        for r in range(1, world):
            np.testing.assert_array_equal(results[r][legacy][0], results[0][legacy][0])


def test_slab_bounds_partition():
    from dvccorr.sharded import slab_bounds
    for H in (1, 7, 8, 9, 32, 64, 128):
        for world in (1, 2, 3, 4, 8):
            if world > H:
                continue
            b = [slab_bounds(H, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == H
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(h1 - h0 for h0, h1 in b) - min(h1 - h0 for h0, h1 in b) <= 1


def _weak_worker(rank, world, port, shape, L, R, q):
    """bench.py --scaling weak: every rank owns its own pair; group=LOCAL must not shard or communicate."""
    import sys
    for p in (REPO, PKG, os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import prng
        from dvccorr.sharded import LOCAL, ShardedCorrBlock
        B, C, H, W, D = shape
        f1 = torch.from_numpy(prng.normal(51 + 10 * rank, shape))
        f2 = torch.from_numpy(prng.normal(52 + 10 * rank, shape))
        coords = torch.from_numpy(prng.flow_coords(53 + 10 * rank, B, H, W, D, 2.0))
        blk = ShardedCorrBlock(f1, f2, H, L, R, False, precision="fp32", backend=TorchCpuRows, group=LOCAL)
        assert (blk.world, blk.rank, blk.h0, blk.h1) == (1, 0, 0, H)
        q.put((rank, blk(coords).numpy()))
    finally:
        dist.destroy_process_group()


def test_weak_scaling_replicas_are_independent():
    from oracle import torch_cpu
    import prng
    world, shape, L, R = 2, (1, 8, 8, 8, 8), 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_weak_worker, args=(r, world, port, shape, L, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B, C, H, W, D = shape
    for r in range(world):
        f1 = torch.from_numpy(prng.normal(51 + 10 * r, shape))
        f2 = torch.from_numpy(prng.normal(52 + 10 * r, shape))
        coords = torch.from_numpy(prng.flow_coords(53 + 10 * r, B, H, W, D, 2.0))
        ref = torch_cpu.corr_lookup(f1, f2, coords, L, R, False).numpy()
        np.testing.assert_allclose(results[r], ref, rtol=0, atol=2e-6 * np.abs(ref).max())
