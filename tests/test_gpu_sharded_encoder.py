"""GPU: the sharded feature encoder feeding the sharded correlation block.

Each rank runs the model's fnet (a RAFT-DVC 1/4 encoder, MediumEncoder, extractor.py:304-412, in the
reference-pinned restatement tests/raftdvc_encoder.py) on its H-slab of the two input volumes
(dvccorr.sharded_encoder.ShardedEncoder: neighbour halo exchange + all-reduced instance-norm statistics),
and hands its feature slabs to ShardedCorrBlock (HipRows: fmap2 all-gathered, this rank's rows built and
looked up on the GPU).  Checked against the whole-volume path the reference runs (fnet([vol0, vol1]) then
CorrBlock, raft_dvc.py:360-420):
  * features: <= 2e-5 of max|ref| (the statistics' fp32 reduction order differs);
  * corr rows: bitwise equal to CorrBlock over the same (assembled) features -- sharding only
    re-partitions independent query rows.
World 1 (group "local") and a 2-rank job on this one device (gloo: the halo planes are staged through the
host; the bench rehearses RCCL's call sites the same way).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

import prng
import raftdvc_encoder as renc

pytestmark = pytest.mark.gpu

FEAT_TOL = 2e-5
S_IN, STRIDE, L, R = 64, 4, 4, 4
S = S_IN // STRIDE


def _problem(dev):
    enc = renc.Encoder("1/4")
    renc.set_params(enc, 4242)
    enc = enc.to(dev).eval()
    v0 = prng.uniform(4243, (1, 1, S_IN, S_IN, S_IN))
    v1 = np.ascontiguousarray(np.roll(v0, (2, -1, 3), axis=(2, 3, 4)))
    coords = prng.flow_coords(4244, 1, S, S, S, 2.0)
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    return enc, t(v0), t(v1), t(coords)


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


def test_world1_encoder_feeds_sharded_block():
    import dvccorr
    from dvccorr.sharded import ShardedCorrBlock
    from dvccorr.sharded_encoder import ShardedEncoder
    dev = torch.device("cuda:0")
    enc, v0, v1, coords = _problem(dev)
    with torch.no_grad():
        f0, f1 = enc(torch.cat([v0, v1])).split(1)               # the whole-volume fnet([vol0, vol1])
        s0, s1 = ShardedEncoder(enc, group="local")([v0, v1], S_IN)
        assert _rel(s0, f0) <= FEAT_TOL and _rel(s1, f1) <= FEAT_TOL
        out = ShardedCorrBlock(s0, s1, S, L, R, precision="bf16", group="local")(coords)
        ref = dvccorr.CorrBlock(s0, s1, L, R, precision="bf16")(coords)
        torch.cuda.synchronize()
    assert torch.equal(out, ref)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "raft-dvc_amd"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dvccorr.sharded import ShardedCorrBlock, slab_bounds
        from dvccorr.sharded_encoder import ShardedEncoder
        dev = torch.device("cuda:0")
        enc, v0, v1, coords = _problem(dev)
        se = ShardedEncoder(enc)
        i0, i1 = se.input_bounds(S_IN)
        h0, h1 = slab_bounds(S, world, rank)
        with torch.no_grad():
            s0, s1 = se([v0[:, :, i0:i1].contiguous(), v1[:, :, i0:i1].contiguous()], S_IN)
            blk = ShardedCorrBlock(s0, s1, S, L, R, precision="bf16")
            out = blk(coords[:, :, h0:h1].contiguous())
            torch.cuda.synchronize()
        # numpy arrays travel as plain pickled bytes: a torch CPU tensor would be handed over as a shared-memory
        # file descriptor, which races this process's exit (EOFError in the parent)
        q.put((rank, s0.cpu().numpy(), s1.cpu().numpy(), out.cpu().numpy()))
    except Exception as e:   # report instead of hanging the parent
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_device():
    import torch.multiprocessing as mp
    import dvccorr
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in range(world):
            r, a, b, o = q.get(timeout=240)
            assert b is not None, f"rank {r}: {a}"
            got[r] = (a, b, o)
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    dev = torch.device("cuda:0")
    enc, v0, v1, coords = _problem(dev)
    s0 = torch.cat([torch.from_numpy(got[r][0]) for r in range(world)], dim=2).to(dev)
    s1 = torch.cat([torch.from_numpy(got[r][1]) for r in range(world)], dim=2).to(dev)
    out = torch.cat([torch.from_numpy(got[r][2]) for r in range(world)], dim=2).to(dev)
    with torch.no_grad():
        f0, f1 = enc(torch.cat([v0, v1])).split(1)
        assert _rel(s0, f0) <= FEAT_TOL and _rel(s1, f1) <= FEAT_TOL
        ref = dvccorr.CorrBlock(s0, s1, L, R, precision="bf16")(coords)
        torch.cuda.synchronize()
    assert torch.equal(out, ref)
