#!/usr/bin/env python3
"""Diagnostics: locate the intermittent k_fused_proj difference -- in the per-query rows (k_fused_proj) or
in their transpose (k_rows_to_channels)?  Explicit workspace, inspected after each call."""
import sys
sys.path.insert(0, "raft-dvc_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch, prng  # noqa: E401
import dvccorr  # noqa: E402
from dvccorr import ops  # noqa: E402
DEV = torch.device("cuda:0")


def poison(val):
    bufs = [torch.full((mb * (1 << 20) // 4,), val, device=DEV) for mb in (1, 3, 7, 16, 40, 100) for _ in range(3)]
    torch.cuda.synchronize()
    del bufs


shape, C, L, r, legacy, B = (12, 10, 16), 64, 3, 2, False, 1
H, W, D = shape
seed = 1900 + H + 3 * W + 7 * D + r
f1 = prng.normal(seed, (2, C, H, W, D))[1:]; f2 = prng.normal(seed + 1, (2, C, H, W, D))[1:]
coords = prng.flow_coords(seed + 2, 2, H, W, D, 2.5)[1:]
K = L * (2 * r + 1) ** 3; bound = 1.0 / np.sqrt(K)
w = prng.uniform(seed + 3, (96, K), -bound, bound); bb = prng.uniform(seed + 4, (96,), -bound, bound)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
t1, t2, tc, tw, tb = T(f1), T(f2), T(coords), T(w), T(bb)
Nq = H * W * D
nws = ops.lib().dvc_lookup_fused_proj_workspace_bytes(B, Nq)
rows_bytes = (B * Nq * 96 * 4 + 255) // 256 * 256
keys_bytes = (Nq * 8 + 255) // 256 * 256
abl = int(sys.argv[1]) if len(sys.argv) > 1 else 0
if abl:
    from dvccorr import _lib
    _lib.set_tuning("fused_ablate", abl)
with torch.no_grad():
    blk = dvccorr.CorrBlockFused(t1, t2, L, r, precision="bf16")
    pw = ops.proj_pack(tw, L, r, False)

    def call(ws):
        out = ops.lookup_fused_proj(blk._q, blk._t, tc.reshape(B, 3, -1), pw, tb, C, H, W, D, L, r, False,
                                    blk._dt, workspace=ws)
        torch.cuda.synchronize()
        rows = ws[nws - rows_bytes:nws].view(torch.float32)[:B * Nq * 96].reshape(B, Nq, 96).clone()
        kout = ws[keys_bytes:2 * keys_bytes].view(torch.int64)[:Nq].clone()
        return out.clone(), rows, kout

    ref = call(torch.zeros((nws,), dtype=torch.uint8, device=DEV))
    stats = {"out": 0, "rows": 0, "kout": 0, "out_not_rows": 0}
    for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
        poison((-7.0, 3.0e4, float("nan"))[it % 3])
        ws = torch.empty((nws,), dtype=torch.uint8, device=DEV)
        got = call(ws)
        do, dr, dk = (not torch.equal(got[0], ref[0])), (not torch.equal(got[1], ref[1])), (not torch.equal(got[2], ref[2]))
        stats["out"] += do; stats["rows"] += dr; stats["kout"] += dk
        if do and not dr:
            stats["out_not_rows"] += 1
        if do or dr or dk:
            msg = f"it {it}: out {do} rows {dr} kout {dk}"
            if dr:
                d = (got[1] - ref[1]).abs()
                qs = torch.nonzero(d.amax(dim=2) > 0)[:, 1]
                msg += f"; {qs.numel()} query rows differ, e.g. q {qs[:8].tolist()}, max {float(d.nan_to_num(1e30).max()):.3e}"
                chans = torch.nonzero(d.amax(dim=(0, 1)) > 0).flatten().tolist()
                qsorted = (ref[2] & 0xffffffff).tolist()
                pos = sorted(qsorted.index(int(qq)) for qq in qs.tolist())
                msg += f"; channels {len(chans)}: {chans[:4]}..{chans[-2:]}; sorted slots {pos}"
            print(msg[:200], flush=True)
    print("fused_ablate", abl, "stats", stats, flush=True)
