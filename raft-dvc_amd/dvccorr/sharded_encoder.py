"""Query-voxel sharding of the feature encoder.

At 256^3 inputs every rank of the sharded correlation block (sharded.py) owns an
H-slab of the feature maps; running the whole feature encoder on every rank
would replicate the encoder's work n times.  ShardedEncoder runs a RAFT-DVC
feature encoder -- BasicEncoder (1/8, extractor.py:142-256), MediumEncoder
(1/4, :304-412) or ShallowEncoder (1/2, :415-523), the same module object the
model holds -- on this rank's H-slab of the input volume and returns this
rank's slab of the feature map, ready for ShardedCorrBlock.

The encoder's layers are interpreted from the module tree (conv1 / norm1 /
relu, layer1..layerK of residual or bottleneck blocks, conv2), so trained
weights are used as they are.  Two exchanges make the slab computation equal
to the whole-volume one:

  * halo planes: before every convolution with a spatial extent along H, each
    rank receives the planes the kernel reaches across its slab boundaries
    from its two neighbours (zeros beyond the volume, as the reference's zero
    padding): one batched point-to-point exchange with rank - 1 and rank + 1
    per convolution (dist.batch_isend_irecv), so a rank's halo traffic does not
    grow with the number of ranks;
  * normalisation statistics: InstanceNorm3d / GroupNorm / training-mode
    BatchNorm3d normalise over the whole volume, so their per-channel sums are
    all-reduced (two passes: mean, then the centred sum of squares, as the
    reference's biased variance).

Scope (forward only): the collectives above carry no autograd, so the encoder
is run for inference -- a call that would need gradients (grad mode on and
the input or any encoder parameter requiring grad) raises, as ShardedCorrBlock
does.  Only encoders whose forward is the reference's conv1 -> norm1 -> relu ->
layers -> conv2 sequence are accepted: BasicEncoder, MediumEncoder and
ShallowEncoder (and subclasses that keep their forward, e.g. LateStrideEncoder,
extractor.py:526); a subclass that overrides forward (ShallowUpEncoder adds a
trilinear x2 upsample, extractor.py:549-566) is refused unless its class sets
`sharded_forward_equivalent = True` itself.  Training-mode norms that track running
statistics are refused (the slab pass would not update them).

Slabs follow sharded.slab_bounds on the feature-map H axis; rank r's input
slab is planes [s * h0, s * h1) of the volume (s = the encoder's total
stride, H divisible by s).  Results equal the whole-volume encoder's up to
the fp32 reduction order of the statistics (tests/test_sharded_encoder.py).
The reference has no distributed code; this is new design.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .sharded import LOCAL, _rank, _world, slab_bounds

__all__ = ["ShardedEncoder", "encoder_stride"]


def _conv_h(m: nn.Conv3d) -> Tuple[int, int, int]:
    """(kernel, stride, padding) of a Conv3d along H (dim 2)."""
    k, s, p = m.kernel_size[0], m.stride[0], m.padding[0]
    if isinstance(p, str):
        raise NotImplementedError(f"string padding {p!r} is not supported")
    return k, s, p


def _blocks(encoder: nn.Module) -> List[nn.Module]:
    out = []
    i = 1
    while hasattr(encoder, f"layer{i}"):
        layer = getattr(encoder, f"layer{i}")
        out.extend(list(layer) if isinstance(layer, nn.Sequential) else [layer])
        i += 1
    return out


def encoder_stride(encoder: nn.Module) -> int:
    """Total downsampling along H of conv1 and every block (8, 4, 2 for the 1/8, 1/4, 1/2 encoders)."""
    s = _conv_h(encoder.conv1)[1]
    for blk in _blocks(encoder):
        convs = [getattr(blk, n) for n in ("conv1", "conv2", "conv3") if hasattr(blk, n)]
        for c in convs:
            s *= _conv_h(c)[1]
    return s * _conv_h(encoder.conv2)[1]


class ShardedEncoder:
    """Run `encoder` on this rank's H-slab.  __call__(volume_slab | [vol0_slab, vol1_slab], H) -> feature slab(s)."""

    #: classes whose forward is the sequence interpreted here (extractor.py:218-256, :386-412, :497-523)
    KNOWN_FORWARDS = ("BasicEncoder", "MediumEncoder", "ShallowEncoder")

    def __init__(self, encoder: nn.Module, group=None):
        for name in ("conv1", "norm1", "conv2"):
            if not hasattr(encoder, name):
                raise TypeError(f"ShardedEncoder: encoder has no {name!r} (expected a RAFT-DVC feature encoder)")
        owner = next((k for k in type(encoder).__mro__ if "forward" in vars(k)), None)
        if not (owner is not None and (owner.__name__ in self.KNOWN_FORWARDS
                                       or vars(owner).get("sharded_forward_equivalent", False))):
            raise NotImplementedError(
                f"ShardedEncoder: {type(encoder).__name__}.forward is defined by "
                f"{getattr(owner, '__name__', None)}, not by one of {self.KNOWN_FORWARDS}; a forward that adds "
                f"steps (e.g. ShallowUpEncoder's x2 upsample) would be skipped by the slab interpreter")
        if getattr(encoder, "training", False) and getattr(encoder, "dropout", None) is not None:
            raise NotImplementedError("ShardedEncoder: dropout in training mode is not supported")
        for m in encoder.modules():
            if isinstance(m, nn.modules.batchnorm._NormBase) and m.training and m.track_running_stats:
                raise NotImplementedError(
                    f"ShardedEncoder: training-mode {type(m).__name__} with track_running_stats would not update "
                    f"its running statistics on the slab pass; call encoder.eval() or disable tracking")
        self.enc = encoder
        self.group = group
        self.world, self.rank = _world(group), _rank(group)
        self.stride = encoder_stride(encoder)
        self._thin = 1.0   # (thinnest rank's slab) / (this rank's slab), set per call

    # ---------------------------------------------------------------- collectives
    def _all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def _peer(self, r: int) -> int:
        """Global rank of group rank r (point-to-point ops address global ranks)."""
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def _halo(self, x: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
        """x with `lo` planes of the previous slab prepended and `hi` of the next appended (zeros at the ends).

        Neighbour exchange: this rank sends its last `lo` planes to rank + 1 and its first `hi` planes to
        rank - 1, and receives the matching planes from them -- four point-to-point ops at most, whatever
        the number of ranks."""
        if lo == 0 and hi == 0:
            return x
        m = max(lo, hi)
        below = x.new_zeros(x.shape[:2] + (lo,) + x.shape[3:])
        above = x.new_zeros(x.shape[:2] + (hi,) + x.shape[3:])
        if self.world > 1:
            # every rank applies the same test (the thinnest slab scales like this one): all raise together
            if x.shape[2] * self._thin < m:
                raise ValueError(f"ShardedEncoder: a slab of {int(x.shape[2] * self._thin)} planes is thinner than "
                                 f"the {m}-plane halo; use fewer ranks for this volume")
            # gloo moves host memory only: device tensors are staged through the host (rehearsals)
            host = x.is_cuda and dist.get_backend(self.group) != "nccl"
            stage = (lambda t: t.cpu()) if host else (lambda t: t.contiguous())
            bl, ab = stage(below), stage(above)
            r, ops = self.rank, []
            if r > 0:
                if hi:
                    ops.append(dist.P2POp(dist.isend, stage(x[:, :, :hi]), self._peer(r - 1), self.group))
                if lo:
                    ops.append(dist.P2POp(dist.irecv, bl, self._peer(r - 1), self.group))
            if r < self.world - 1:
                if lo:
                    ops.append(dist.P2POp(dist.isend, stage(x[:, :, x.shape[2] - lo:]), self._peer(r + 1),
                                          self.group))
                if hi:
                    ops.append(dist.P2POp(dist.irecv, ab, self._peer(r + 1), self.group))
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            if host:
                below, above = bl.to(x.device), ab.to(x.device)
            else:
                below, above = bl, ab
        return torch.cat([below, x, above], dim=2)

    # ---------------------------------------------------------------- layers
    def _conv(self, m: nn.Conv3d, x: torch.Tensor) -> torch.Tensor:
        k, s, p = _conv_h(m)
        if m.dilation[0] != 1 or m.groups != 1:
            raise NotImplementedError("ShardedEncoder: dilated / grouped convolutions are not supported")
        n_out = x.shape[2] // s
        lo, hi = p, max(k - p - s, 0)
        xh = self._halo(x, lo, hi)
        pad = (0,) + tuple(m.padding[1:])
        y = F.conv3d(xh, m.weight, m.bias, stride=m.stride, padding=pad)
        return y[:, :, :n_out]

    def _norm(self, m: nn.Module, x: torch.Tensor) -> torch.Tensor:
        if isinstance(m, nn.Identity):
            return x
        if isinstance(m, nn.InstanceNorm3d):
            if m.track_running_stats and not m.training:
                return F.instance_norm(x, m.running_mean, m.running_var, m.weight, m.bias, False, 0.0, m.eps)
            y = self._normalise(x, dims=(2, 3, 4), eps=m.eps)
            return y if not m.affine else y * m.weight.view(1, -1, 1, 1, 1) + m.bias.view(1, -1, 1, 1, 1)
        if isinstance(m, nn.BatchNorm3d):
            if not m.training and m.track_running_stats:
                return F.batch_norm(x, m.running_mean, m.running_var, m.weight, m.bias, False, 0.0, m.eps)
            y = self._normalise(x.transpose(0, 1), dims=(1, 2, 3, 4), eps=m.eps).transpose(0, 1)
            return y if not m.affine else y * m.weight.view(1, -1, 1, 1, 1) + m.bias.view(1, -1, 1, 1, 1)
        if isinstance(m, nn.GroupNorm):
            B, C = x.shape[:2]
            g = x.reshape(B, m.num_groups, C // m.num_groups, *x.shape[2:])
            y = self._normalise(g, dims=(2, 3, 4, 5), eps=m.eps).reshape(x.shape)
            return y if not m.affine else y * m.weight.view(1, -1, 1, 1, 1) + m.bias.view(1, -1, 1, 1, 1)
        raise NotImplementedError(f"ShardedEncoder: normalisation {type(m).__name__} is not supported")

    def _normalise(self, x: torch.Tensor, dims, eps: float) -> torch.Tensor:
        """(x - mean) / sqrt(var + eps) with mean / biased var over `dims` of the WHOLE volume (all ranks)."""
        n = torch.tensor(float(torch.tensor([x.shape[d] for d in dims]).prod()), device=x.device, dtype=torch.float64)
        n = self._all_reduce(n.clone())
        s = self._all_reduce(x.double().sum(dim=dims, keepdim=True))
        mean = (s / n).to(x.dtype)
        c = x - mean
        ss = self._all_reduce((c.double() * c.double()).sum(dim=dims, keepdim=True))
        var = (ss / n).to(x.dtype)
        return c / torch.sqrt(var + eps)

    def _block(self, blk: nn.Module, x: torch.Tensor) -> torch.Tensor:
        if hasattr(blk, "conv3"):   # BottleneckBlock3D (extractor.py:72-141)
            y = F.relu(self._norm(blk.norm1, self._conv(blk.conv1, x)))
            y = F.relu(self._norm(blk.norm2, self._conv(blk.conv2, y)))
            y = self._norm(blk.norm3, self._conv(blk.conv3, y))
        else:                       # ResidualBlock3D (extractor.py:12-70)
            y = F.relu(self._norm(blk.norm1, self._conv(blk.conv1, x)))
            y = self._norm(blk.norm2, self._conv(blk.conv2, y))
        if blk.downsample is not None:
            conv, norm = blk.downsample[0], blk.downsample[1]
            x = self._norm(norm, self._conv(conv, x))
        return F.relu(y + x)

    def forward_slab(self, x: torch.Tensor) -> torch.Tensor:
        e = self.enc
        x = F.relu(self._norm(e.norm1, self._conv(e.conv1, x)))
        for blk in _blocks(e):
            x = self._block(blk, x)
        return self._conv(e.conv2, x)

    def input_bounds(self, H: int) -> Tuple[int, int]:
        """This rank's input planes [s h0, s h1) for a volume of H planes (H divisible by the stride)."""
        if H % self.stride:
            raise ValueError(f"ShardedEncoder: H={H} is not a multiple of the encoder stride {self.stride}")
        h0, h1 = slab_bounds(H // self.stride, self.world, self.rank)
        return self.stride * h0, self.stride * h1

    def __call__(self, x: Union[torch.Tensor, Sequence[torch.Tensor]], H: Optional[int] = None):
        """x: this rank's input slab (B, C, s (h1 - h0), W, D), or [vol0_slab, vol1_slab] (the fnet call,
        extractor.py:397-410: both volumes through one pass, split after).  H: full input H (checks the slab)."""
        is_list = isinstance(x, (list, tuple))
        xs = torch.cat(list(x), dim=0) if is_list else x
        if torch.is_grad_enabled() and (xs.requires_grad or any(p.requires_grad for p in self.enc.parameters())):
            raise NotImplementedError(
                "ShardedEncoder is forward-only (its halo and statistics exchanges carry no autograd): run it "
                "under torch.no_grad() / inference_mode, or use the whole-volume encoder for training")
        if self.world > 1:   # the thinnest slab, for the halo check every rank makes alike
            t = torch.tensor([xs.shape[2]], dtype=torch.float64, device=xs.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            self._thin = float(t.item()) / xs.shape[2]
        if H is not None:
            i0, i1 = self.input_bounds(H)
            if xs.shape[2] != i1 - i0:
                raise ValueError(f"rank {self.rank}: input slab has {xs.shape[2]} planes, expected {i1 - i0}")
        y = self.forward_slab(xs)
        if is_list:
            return tuple(torch.split(y, [t.shape[0] for t in x], dim=0))
        return y
