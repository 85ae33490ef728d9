"""Portable counter-based PRNG for test inputs (bit-identical on any machine).

Golden fixtures store only seeds and shapes for their inputs; the GPU box
regenerates the same float32 inputs with this module, so no torch/numpy RNG
parity across machines is needed.  Only integer arithmetic and exact
float64 sums are used (no transcendental functions), so results do not
depend on libm or SIMD paths.

    uniform24(seed, n)  -> float64 k * 2**-24, k in [0, 2**24)
    normal(seed, shape) -> float32, Irwin-Hall(12) - 6  (mean 0, var 1)
"""
from __future__ import annotations

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_SEEDMIX = np.uint64(0xD1B54A32D192ED03)


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _stream(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        base = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) * _SEEDMIX
    idx = np.arange(n, dtype=np.uint64)
    return _splitmix(idx ^ base)


def uniform24(seed: int, n: int) -> np.ndarray:
    """n float64 values k * 2**-24 in [0, 1), exactly representable in fp32."""
    return (_stream(seed, n) >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


def uniform(seed: int, shape, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    n = int(np.prod(shape))
    u = uniform24(seed, n)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def normal(seed: int, shape) -> np.ndarray:
    """Approximately N(0,1) float32 (sum of 12 uniforms minus 6; exact in fp64)."""
    n = int(np.prod(shape))
    u = uniform24(seed, 12 * n).reshape(12, n)
    s = u[0].copy()
    for k in range(1, 12):
        s += u[k]
    return (s - 6.0).astype(np.float32).reshape(shape)


def identity_coords(B: int, H: int, W: int, D: int) -> np.ndarray:
    """coords_grid_3d (reference corr.py:71-99): (B, 3, H, W, D), channel c = index on axis c."""
    g = np.stack(np.meshgrid(np.arange(H), np.arange(W), np.arange(D), indexing="ij"), axis=0)
    return np.broadcast_to(g.astype(np.float32), (B, 3, H, W, D)).copy()


def flow_coords(seed: int, B: int, H: int, W: int, D: int, max_flow: float) -> np.ndarray:
    """Identity grid + U(-max_flow, max_flow) per channel (test_corr_equivalence.py:52-76 pattern)."""
    base = identity_coords(B, H, W, D).astype(np.float64)
    u = uniform24(seed, B * 3 * H * W * D).reshape(B, 3, H, W, D)
    return (base + (2.0 * u - 1.0) * max_flow).astype(np.float32)
