import sys, os
sys.path.insert(0, "/root/repo/raft-dvc_amd"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
import numpy as np, torch, prng, dvccorr
DEV = torch.device("cuda:0")
def conv(seed, L, r):
    K = L * (2 * r + 1) ** 3; bound = 1.0 / np.sqrt(K)
    return prng.uniform(seed, (96, K), -bound, bound), prng.uniform(seed + 1, (96,), -bound, bound)
torch.set_grad_enabled(False)
for (shape, C, L, r, B) in [((12,10,16),64,3,2,2), ((12,10,16),64,3,2,1), ((12,10,16),32,3,2,1), ((12,12,12),64,3,2,1), ((12,10,16),64,1,2,1), ((8,8,8),64,1,2,1), ((16,16,16),64,1,3,1), ((16,16,16),64,1,4,1), ((16,16,16),64,1,1,1)]:
    H, W, D = shape
    seed = 1900 + H + 3 * W + 7 * D + r
    f1 = prng.normal(seed, (B, C, H, W, D)); f2 = prng.normal(seed + 1, (B, C, H, W, D))
    coords = prng.flow_coords(seed + 2, B, H, W, D, 2.5)
    w, b = conv(seed + 3, L, r)
    t1, t2, tc, tw, tb = [torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in (f1, f2, coords, w, b)]
    out = dvccorr.CorrBlockFused(t1, t2, L, r, precision="bf16").lookup_convc1(tc, tw, tb)
    mat = dvccorr.CorrBlock(t1, t2, L, r, precision="bf16").lookup_convc1(tc, tw, tb)
    d = (out - mat).abs()
    err = float(d.max() / mat.abs().max())
    bad = (d.amax(1) > 1e-3 * float(mat.abs().max()))
    idx = bad.nonzero()[:8].tolist()
    print(shape, C, L, r, B, "err", f"{err:.2e}", "bad voxels", int(bad.sum()), idx, flush=True)
