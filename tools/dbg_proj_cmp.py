#!/usr/bin/env python3
"""Determinism stress of the two convc1-fused lookups on the test_gpu_proj_fused shapes: each kernel's
output compared bitwise with its own first output over many calls (allocator state perturbed between
calls), and the two kernels compared with each other.  Diagnostics only."""
import sys
sys.path.insert(0, "raft-dvc_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch, prng  # noqa: E401
import dvccorr  # noqa: E402
DEV = torch.device("cuda:0")
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
for (shape, C, L, r, legacy, B) in [((12, 10, 16), 64, 3, 2, False, 2), ((9, 7, 5), 32, 2, 1, False, 1),
                                    ((11, 9, 13), 128, 3, 4, False, 1), ((16, 16, 16), 32, 4, 3, False, 1)]:
    H, W, D = shape
    seed = 1900 + H + 3 * W + 7 * D + r
    f1 = prng.normal(seed, (B, C, H, W, D)); f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, 2.5)
    K = L * (2 * r + 1) ** 3; bound = 1.0 / np.sqrt(K)
    w = prng.uniform(seed + 3, (96, K), -bound, bound); b = prng.uniform(seed + 4, (96,), -bound, bound)
    t1, t2, tc, tw, tb = [torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in (f1, f2, coords, w, b)]
    fo = fm = None
    nbad_o = nbad_m = 0
    junk = []
    for it in range(iters):
        junk.append(torch.randn(int(1e5) * (1 + it % 7), device=DEV))   # perturb the allocator / memory contents
        if len(junk) > 5:
            junk.pop(0)
        out = dvccorr.CorrBlockFused(t1, t2, L, r, legacy_wd_swap=legacy, precision="bf16").lookup_convc1(tc, tw, tb)
        mat = dvccorr.CorrBlock(t1, t2, L, r, legacy_wd_swap=legacy, precision="bf16").lookup_convc1(tc, tw, tb)
        torch.cuda.synchronize()
        if fo is None:
            fo, fm = out.clone(), mat.clone()
            print(shape, "first: out~mat", float((out - mat).abs().max() / mat.abs().max()), flush=True)
            continue
        if not torch.equal(out, fo):
            nbad_o += 1
            d = (out - fo).abs()
            idx = torch.nonzero(d > 0)
            print(f"  it {it}: FUSED differs from its first output: max {float(d.max()):.3e}, {idx.shape[0]} entries, "
                  f"e.g. {idx[:6].tolist()}", flush=True)
        if not torch.equal(mat, fm):
            nbad_m += 1
            d = (mat - fm).abs()
            idx = torch.nonzero(d > 0)
            print(f"  it {it}: MATERIALISED differs from its first output: max {float(d.max()):.3e}, "
                  f"{idx.shape[0]} entries, e.g. {idx[:6].tolist()}", flush=True)
    print(shape, f"iters {iters}: fused nondeterministic {nbad_o}, materialised nondeterministic {nbad_m}", flush=True)
