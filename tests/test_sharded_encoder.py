"""CPU, multi-process (gloo): the sharded feature encoder (dvccorr.sharded_encoder).

Each rank runs a RAFT-DVC feature encoder on its H-slab of the input volume (halo planes and
normalisation statistics exchanged) and must produce its slab of the whole-volume encoder's output.
The encoders are tests/raftdvc_encoder.py's restatement of extractor.py, pinned against the reference's
own outputs (tests/golden/encoder_*.npz, gen_encoder_golden.py).  World sizes 1, 2 and 3 (uneven slabs);
the 1/8, 1/4 and 1/2 encoders; the fnet list call [vol0, vol1].
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import prng
import raftdvc_encoder as renc
from conftest import PKG, REPO, load_golden

TOL = 2e-5


def _encoder(tag):
    g = load_golden(f"encoder_{tag}.npz")
    kind = {"1_8": "1/8", "1_4": "1/4", "1_2": "1/2"}[tag]
    enc = renc.Encoder(kind).eval()
    renc.set_params(enc, int(g["seed0"][0]))
    x = torch.from_numpy(prng.uniform(int(g["in_seed"][0]), tuple(int(v) for v in g["in_shape"])))
    return enc, x, g["out"]


@pytest.mark.parametrize("tag", ["1_8", "1_4", "1_2"])
def test_restated_encoder_matches_reference(tag):
    enc, x, ref = _encoder(tag)
    with torch.no_grad():
        out = enc(x).numpy()
    assert np.abs(out - ref).max() <= 1e-6 * np.abs(ref).max()


@pytest.mark.parametrize("tag", ["1_8", "1_4", "1_2"])
def test_single_rank_equals_encoder(tag):
    from dvccorr.sharded_encoder import ShardedEncoder, encoder_stride
    enc, x, ref = _encoder(tag)
    assert encoder_stride(enc) == {"1_8": 8, "1_4": 4, "1_2": 2}[tag]
    with torch.no_grad():
        out = ShardedEncoder(enc, group="local")(x, x.shape[2]).numpy()
    assert np.abs(out - ref).max() <= TOL * np.abs(ref).max()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (REPO, PKG, os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dvccorr.sharded_encoder import ShardedEncoder
        res = {}
        for tag in ("1_8", "1_4", "1_2"):
            enc, x, _ = _encoder(tag)
            se = ShardedEncoder(enc)
            i0, i1 = se.input_bounds(x.shape[2])
            x2 = torch.roll(x, 3, dims=4)
            with torch.no_grad():
                a, b = se([x[:, :, i0:i1], x2[:, :, i0:i1]], x.shape[2])
            res[tag] = (a.numpy(), b.numpy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_encoder_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for tag in ("1_8", "1_4", "1_2"):
        enc, x, ref = _encoder(tag)
        with torch.no_grad():
            ref2 = enc(torch.roll(x, 3, dims=4)).numpy()
        a = np.concatenate([got[r][tag][0] for r in range(world)], axis=2)
        b = np.concatenate([got[r][tag][1] for r in range(world)], axis=2)
        assert a.shape == ref.shape
        assert np.abs(a - ref).max() <= TOL * np.abs(ref).max(), (tag, world)
        assert np.abs(b - ref2).max() <= TOL * np.abs(ref2).max(), (tag, world)


def test_thin_slab_raises():
    from dvccorr.sharded_encoder import ShardedEncoder
    enc, x, _ = _encoder("1_8")
    se = ShardedEncoder(enc, group="local")
    with torch.no_grad(), pytest.raises(ValueError, match="multiple of the encoder stride"):
        se(x[:, :, :12], 12)


def test_forward_only_guard():
    """The halo / statistics exchanges carry no autograd: a call that would need gradients raises."""
    from dvccorr.sharded_encoder import ShardedEncoder
    enc, x, _ = _encoder("1_4")
    se = ShardedEncoder(enc, group="local")
    with pytest.raises(NotImplementedError, match="forward-only"):
        se(x, x.shape[2])                       # encoder parameters require grad
    with torch.no_grad():
        se(x, x.shape[2])


def test_refuses_overridden_forward_and_tracked_training_norms():
    """A subclass that changes forward (the reference's ShallowUpEncoder upsamples x2, extractor.py:549-566)
    is refused; one that keeps it (LateStrideEncoder, extractor.py:526) is accepted; training-mode norms
    tracking running statistics are refused."""
    from dvccorr.sharded_encoder import ShardedEncoder
    enc, _, _ = _encoder("1_2")

    class UpEncoder(type(enc)):
        def forward(self, x):
            return torch.nn.functional.interpolate(super().forward(x), scale_factor=2.0, mode="trilinear")

    class SameForward(type(enc)):
        pass

    up = UpEncoder("1/2")
    with pytest.raises(NotImplementedError, match="forward is defined by UpEncoder"):
        ShardedEncoder(up, group="local")
    ShardedEncoder(SameForward("1/2"), group="local")
    bn = renc.Encoder("1/4")
    bn.norm1 = torch.nn.BatchNorm3d(32)
    bn.train()
    with pytest.raises(NotImplementedError, match="running statistics"):
        ShardedEncoder(bn, group="local")
    ShardedEncoder(bn.eval(), group="local")
