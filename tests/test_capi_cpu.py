"""CPU: the C-ABI library loads, exports every declared symbol, and its host
logic (geometry, validation, error mapping) behaves like the reference.
No compute call is made (no GPU here)."""
from __future__ import annotations

import ctypes
import os
import re

import pytest
import torch

from conftest import REPO


def _header_functions():
    txt = open(os.path.join(REPO, "include", "dvccorr.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dvc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from dvccorr import _lib
    L = _lib.lib()
    declared = _header_functions()
    assert len(declared) >= 13
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib.EXPORTED)
    assert L.dvc_abi_version() == 3
    assert b"gfx950" in L.dvc_version()


def test_library_is_gfx950_code_object():
    from dvccorr import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("shape,L,expect", [
    ((32, 32, 32), 4, [(32, 32, 32), (16, 16, 16), (8, 8, 8), (4, 4, 4)]),
    ((16, 16, 16), 4, [(16, 16, 16), (8, 8, 8), (4, 4, 4), (2, 2, 2)]),
    ((8, 8, 8), 4, [(8, 8, 8), (4, 4, 4), (2, 2, 2), (1, 1, 1)]),
    ((9, 7, 8), 3, [(9, 7, 8), (4, 3, 4), (2, 1, 2)]),
    ((128, 128, 128), 2, [(128, 128, 128), (64, 64, 64)]),
])
def test_layout_geometry(shape, L, expect):
    from dvccorr import layout
    lay = layout(*shape, L, 128)
    assert lay.levels() == expect
    off = 0
    for l, (h, w, d) in enumerate(expect):
        assert lay.Dp[l] % 8 == 0 and lay.Dp[l] >= d
        assert lay.offset[l] == off
        assert lay.level_elems[l] == h * w * lay.Dp[l]
        assert lay.zero_level[l] == int(min(h, w, d) == 1)
        off += lay.level_elems[l]
    assert lay.row_elems == off and lay.row_stride % 128 == 0 and lay.row_stride >= off
    assert lay.c_pad == 128


def test_layout_raises_where_reference_raises():
    from dvccorr import layout
    with pytest.raises(RuntimeError):
        layout(8, 8, 2, 3)          # (4,4,1) cannot be pooled again (avg_pool3d error)
    with pytest.raises(RuntimeError):
        layout(8, 8, 8, 5)
    layout(8, 8, 2, 2)


def test_bf16_row_bytes_for_baseline_configs():
    """pyramid elements N * P_L (unpadded) for configs #2-#4."""
    from dvccorr import layout
    for S, N, PL in ((16, 4096, 1.917e7), (32, 32768, 1.227e9), (64, 262144, 7.85e10)):
        lay = layout(S, S, S, 4, 128)
        unpadded = sum(h * w * d for (h, w, d) in lay.levels())
        assert abs(N * unpadded - PL) / PL < 0.001
        assert lay.row_elems <= 1.02 * unpadded     # z padding to 8 costs <= 2 %


def test_validation_errors_without_gpu():
    """Argument checks run before any HIP call and map to ValueError."""
    from dvccorr import _lib
    L = _lib.lib()
    rc = L.dvc_corr_lookup(None, None, None, 1, 8, 2, 2, 2, 1, 4, 0, 0, None)
    assert rc == _lib.DVC_ERR_INVALID
    with pytest.raises(ValueError, match="null pointer"):
        _lib.check(rc)
    rc = L.dvc_corr_build(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 8, 32, 8, 8, 8, 1,
                          _lib.DVC_BF16, _lib.DVC_BF16, 64, 512, None)
    assert rc == _lib.DVC_ERR_INVALID       # column range must start on a 128 boundary
    rc = L.dvc_corr_lookup(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 8, 8, 8, 8, 1, 4, 7,
                           0, None)
    assert rc == _lib.DVC_ERR_INVALID       # convention
    assert L.dvc_lookup_fused_workspace_bytes(1, 100000, 2, 4) == 65536 * 10 * 10 * 12 * 4


def test_pack_targets_gathered_validation_without_gpu():
    """dvc_pack_targets_gathered's host checks (before any HIP call): null pointers, world outside [1, H] and a bad
    dtype are invalid; more than four levels (the single-pass pack only) is unsupported."""
    from dvccorr import _lib
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    assert L.dvc_pack_targets_gathered(None, 2, p, 1, 16, 32, 32, 32, 4, _lib.DVC_BF16, None) == _lib.DVC_ERR_INVALID
    assert L.dvc_pack_targets_gathered(p, 0, p, 1, 16, 32, 32, 32, 4, _lib.DVC_BF16, None) == _lib.DVC_ERR_INVALID
    assert L.dvc_pack_targets_gathered(p, 33, p, 1, 16, 32, 32, 32, 4, _lib.DVC_BF16, None) == _lib.DVC_ERR_INVALID
    assert L.dvc_pack_targets_gathered(p, 2, p, 1, 16, 32, 32, 32, 4, 7, None) == _lib.DVC_ERR_INVALID
    assert L.dvc_pack_targets_gathered(p, 2, p, 1, 16, 64, 64, 64, 5, _lib.DVC_BF16, None) == _lib.DVC_ERR_UNSUPPORTED


def test_product_path_refuses_cpu_tensors():
    import dvccorr
    f = torch.randn(1, 16, 8, 8, 8)
    with pytest.raises(RuntimeError, match="MI355X"):
        dvccorr.CorrBlock(f, f, 2, 4)
    with pytest.raises(RuntimeError, match="MI355X"):
        dvccorr.CorrBlockFused(f, f, 2, 4)


def test_reference_style_argument_errors():
    import dvccorr
    f = torch.randn(1, 16, 8, 8, 8)
    with pytest.raises(ValueError):
        dvccorr.CorrBlock(f, torch.randn(1, 16, 8, 8, 4))
    with pytest.raises(ValueError):
        dvccorr.CorrBlockOnTheFly(f, f, chunk_size=0)
    with pytest.raises(ValueError):
        dvccorr.make_corr_block("mi355x", f, f, sampler_version=3)
    with pytest.raises(RuntimeError, match="MI355X"):   # grad-tracking maps: same refusal of CPU tensors
        dvccorr.CorrBlock(f.clone().requires_grad_(True), f)


def test_backward_validation_without_gpu():
    """dvc_corr_backward's host checks: null pointers -> ValueError; unsupported radius -> NotImplementedError."""
    from dvccorr import _lib
    L = _lib.lib()
    p = ctypes.c_void_p(16)
    rc = L.dvc_corr_backward(None, p, p, p, p, p, p, 1, 512, 16, 8, 8, 8, 2, 4, 0, 0, None)
    assert rc == _lib.DVC_ERR_INVALID
    rc = L.dvc_corr_backward(p, p, p, p, p, p, p, 1, 512, 16, 8, 8, 8, 2, 9, 0, 0, None)
    assert rc == _lib.DVC_ERR_UNSUPPORTED
    with pytest.raises(NotImplementedError, match="radius"):
        _lib.check(rc)
    # legacy convention with W != D is supported: level 0 of (8, 8, 4) at r = 4 has an 11 x 22 x 7 window box
    # (2r+3, ceil(8 * 7/3) + 3, ceil(8 * 3/7) + 3), and the workspace covers either convention
    nws_wd = L.dvc_corr_backward_workspace_bytes(1, 256, 16, 8, 8, 4, 2, 4)
    assert nws_wd >= 256 * (11 * 22 * 7) * 4
    # workspace: window gradients (B*L*Nq*(2r+2)^3 x 4 bytes) + two partial dQ + dT + every level's keys + cell
    # starts + sort scratch + the MFMA path's query and target tiles (4 KB per 8-aligned start: twice the bf16
    # rows; twice again for the fp32 blocks' hi and lo tiles, round 4) -- ~265 MB above the window gradients at #3
    nws = L.dvc_corr_backward_workspace_bytes(1, 32768, 128, 32, 32, 32, 4, 4)
    assert nws >= 4 * 32768 * 1000 * 4 and nws < 4 * 32768 * 1000 * 4 + 300 * 2 ** 20
    # the dtype's own workspace: fp32 = the dtype-less query (hi + lo tiles); bf16 / fp16 without the lo
    # tiles: ntq = L*Nq/8 + 1 query tiles and B * H*W*(D/8) target tiles per level of 4 KB each, ~88 MB at #3
    f32 = L.dvc_corr_backward_workspace_bytes_dtype(1, 32768, 128, 32, 32, 32, 4, 4, _lib.DVC_F32)
    assert f32 == nws
    tiles = (4 * 32768 // 8 + 1 + sum((32 >> l) ** 2 * max(1, (32 >> l) // 8) for l in range(4))) * 4096
    for dt in (_lib.DVC_BF16, _lib.DVC_F16):
        low = L.dvc_corr_backward_workspace_bytes_dtype(1, 32768, 128, 32, 32, 32, 4, 4, dt)
        assert 0 <= nws - low - tiles < 4096, (nws - low, tiles)
    assert L.dvc_corr_backward_workspace_bytes_dtype(1, 32768, 128, 32, 32, 32, 4, 4, 7) == 0


def test_backward_path_selection_without_gpu():
    """Which gradient kernels dvc_corr_backward runs (pure host): every operand dtype (bf16, fp16 = the AMP pyramid,
    fp32 as bf16 hi/lo pairs) on the matrix cores while k_grad_q_mfma's 32-bit buffer offsets cover the volume;
    volumes past that range (a 160^3 level-0 fmap: 160 * 160 * 20 target tiles of 4 KB per (batch, channel group) exceed
    2^31 bytes), on the 64-bit-addressed VALU kernels -- never a descriptor read past its range."""
    from dvccorr import _lib
    L = _lib.lib()
    for dt in (_lib.DVC_BF16, _lib.DVC_F16):
        assert L.dvc_corr_backward_mfma(1, 32768, 128, 32, 32, 32, 4, 4, 0, dt) == 1    # config #3
        assert L.dvc_corr_backward_mfma(1, 4096, 128, 16, 16, 16, 4, 4, 1, dt) == 1     # config #2, legacy
        assert L.dvc_corr_backward_mfma(1, 160 ** 3, 128, 160, 160, 160, 4, 4, 0, dt) == 0
        assert L.dvc_corr_backward_mfma(1, 128 * 128 * 256, 128, 128, 128, 256, 4, 4, 0, dt) == 0
        assert L.dvc_corr_backward_mfma(1, 64 ** 3, 128, 64, 64, 64, 4, 4, 0, dt) == 1   # config #4's fmaps
    # fp32 operands (round 4): split into bf16 hi/lo tiles on the same kernels; tuning "bwd_mfma" 0 = VALU for all
    assert L.dvc_corr_backward_mfma(1, 32768, 128, 32, 32, 32, 4, 4, 0, _lib.DVC_F32) == 1
    assert L.dvc_set_tuning(b"bwd_mfma", 0) == 0
    try:
        for dt in (_lib.DVC_F32, _lib.DVC_BF16, _lib.DVC_F16):
            assert L.dvc_corr_backward_mfma(1, 32768, 128, 32, 32, 32, 4, 4, 0, dt) == 0
    finally:
        L.dvc_set_tuning(b"bwd_mfma", 1)
    assert L.dvc_corr_backward_mfma(1, 32768, 128, 32, 32, 32, 4, 9, 0, _lib.DVC_BF16) == 0   # radius outside 1..6


def test_backward_gout64_bound_without_gpu():
    """k_win_grad_pairs addresses one output-gradient row ((2r+1)^2 channels of Nq floats) through a buffer
    descriptor with 32-bit offsets; rows past 2^31 - 1 bytes (Nq > ~6.6 M at r = 4, ~3.2 M at r = 6) switch to the
    64-bit-addressed instance instead of reading zeros past the range."""
    from dvccorr import _lib
    L = _lib.lib()
    for r in range(1, 7):
        n2 = (2 * r + 1) ** 2
        edge = (0x7FFFFFFF - 256) // (4 * n2)          # the largest Nq whose row still fits
        assert L.dvc_corr_backward_gout64(edge, r) == 0
        assert L.dvc_corr_backward_gout64(edge + 1, r) == 1
    assert L.dvc_corr_backward_gout64(32768, 4) == 0            # config #3
    assert L.dvc_corr_backward_gout64(188 ** 3, 4) == 1         # a 188^3 fmap at r = 4
    assert L.dvc_corr_backward_gout64(150 ** 3, 6) == 1         # 3.4 M queries at r = 6


def test_coords_grid_matches_reference_fixture():
    import numpy as np
    import prng
    import dvccorr
    g = dvccorr.coords_grid_3d(2, 3, 4, 5, torch.device("cpu"))
    np.testing.assert_array_equal(g.numpy(), prng.identity_coords(2, 3, 4, 5))


def test_precision_policy_host_logic(monkeypatch):
    """Explicit precision > DVCCORR_PRECISION > AMP (CUDA autocast, GPU-tested) > input dtype."""
    import dvccorr
    monkeypatch.delenv("DVCCORR_PRECISION", raising=False)
    f32, b16 = torch.zeros(1), torch.zeros(1, dtype=torch.bfloat16)
    assert dvccorr.resolve_precision(f32, None) == "fp32"
    assert dvccorr.resolve_precision(b16, None) == "bf16"
    assert dvccorr.resolve_precision(torch.zeros(1, dtype=torch.float16), None) == "fp16"
    assert dvccorr.resolve_precision(f32, "bf16") == "bf16"
    assert dvccorr.resolve_precision(f32, "float16") == "fp16"
    monkeypatch.setenv("DVCCORR_PRECISION", "bf16")
    assert dvccorr.resolve_precision(f32, None) == "bf16"
    assert dvccorr.resolve_precision(b16, "fp32") == "fp32"
    with pytest.raises(ValueError):
        dvccorr.resolve_precision(f32, "fp8")


@pytest.mark.parametrize("shape,L,expect", [
    ((32, 32, 32), 4, 0b0001),     # level 0 (Dp 32, W 32): bricked; level 1 (16^3): 32-byte z-rows, linear
    ((64, 64, 64), 4, 0b0011),     # levels 0 and 1
    ((64, 36, 64), 4, 0b0000),     # W % 8 != 0 at level 0; level 1 W = 18
    ((16, 16, 16), 4, 0b0000),     # no level with a 64-byte z-row
    ((32, 40, 33), 3, 0b0001),     # Dp 40 >= 32 (D 33 padded)
])
def test_bricked_levels(shape, L, expect):
    """DVC_BRICKED stores exactly the levels with Dp >= 32 and W % 8 == 0 in (1, 8, 8) bricks (host function),
    and the brick slots of such a level are a permutation of its linear slots."""
    from dvccorr import _lib
    from dvccorr.corr_block import brick_index
    lay = _lib.layout(*shape, L, 32)
    assert _lib.bricked_levels(lay) == expect
    for l, (h, w, d) in enumerate(lay.levels()):
        if (expect >> l) & 1:
            idx = brick_index(h, w, lay.Dp[l], torch.device("cpu"))
            assert torch.equal(torch.sort(idx).values, torch.arange(h * w * lay.Dp[l]))


def test_brick_min_dp_knob():
    """Tuning "brick_min_dp" (round 6 A/B: level 1 of config #3 in (1, 8, 8) bricks too) lowers the bricked-level
    threshold to Dp >= 16 for every layout decided after it, is refused for other values, and the product default
    (32) comes back; the knob is process-global like every dvc_set_tuning key."""
    import threading
    from dvccorr import _lib
    lay = _lib.layout(32, 32, 32, 4, 32)
    assert _lib.bricked_levels(lay) == 0b0001
    seen = []
    try:
        _lib.set_tuning("brick_min_dp", 16)
        t = threading.Thread(target=lambda: seen.append(_lib.bricked_levels(_lib.layout(32, 32, 32, 4, 32))))
        t.start()
        t.join()
        assert _lib.bricked_levels(lay) == 0b0011
        assert seen == [0b0011], "the knob did not reach another host thread"
        with pytest.raises(ValueError):   # (DVC_ERR_INVALID)
            _lib.set_tuning("brick_min_dp", 8)
    finally:
        _lib.set_tuning("brick_min_dp", 32)
    assert _lib.bricked_levels(lay) == 0b0001


def test_lookup_stretch_knob():
    """Tuning "lookup_stretch" (round 6): 1 (default) routes legacy W != D levels to k_lookup_stretch (and the on-the-fly
    path to its window boxes), 0 to the per-output generic kernels; other values are refused.  (The GPU tests compare
    the two bit for bit, tests/test_gpu_stretch.py.)"""
    from dvccorr import _lib
    try:
        _lib.set_tuning("lookup_stretch", 0)
        _lib.set_tuning("lookup_stretch", 1)
        with pytest.raises(ValueError):   # (DVC_ERR_INVALID)
            _lib.set_tuning("lookup_stretch", 2)
        _lib.set_tuning("bwd_stretch", 0)
        with pytest.raises(ValueError):
            _lib.set_tuning("bwd_stretch", 3)
    finally:
        _lib.set_tuning("lookup_stretch", 1)
        _lib.set_tuning("bwd_stretch", 1)


def test_brick_flag_policy(monkeypatch):
    """The materialised block bricks its wide levels only for the tile kernel's cases."""
    from dvccorr import _lib
    from dvccorr.corr_block import brick_flag
    lay = _lib.layout(32, 32, 32, 4, 128)
    assert brick_flag(lay, 4, False, True) == _lib.DVC_BRICKED
    assert brick_flag(lay, 4, False, False) == 0          # pooled build / gradients: linear
    assert brick_flag(lay, 4, False, True, bricked=False) == 0
    assert brick_flag(lay, 7, False, True) == 0           # radius outside the tile kernel: the walk
    assert brick_flag(_lib.layout(32, 32, 32, 5, 128), 4, False, True) == 0   # > 4 levels: per-level pack
    assert brick_flag(_lib.layout(32, 32, 40, 4, 128), 4, True, True) == 0    # legacy W != D on a bricked level
    monkeypatch.setenv("DVCCORR_BRICKED", "0")
    assert brick_flag(lay, 4, False, True) == 0
