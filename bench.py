#!/usr/bin/env python3
"""Benchmark of the RAFT-DVC correlation hot path on MI355X.

Metric (BASELINE.json): corr build+lookup voxel-queries/s, 128^3 pair, 1/4
encoder (32^3 x 128-channel feature maps), L=4, r=4, bf16-MFMA build, fp32
lookup.  One step = one RAFTDVC forward's worth of correlation work:
    [N>1: all-gather of the fmap2 slabs over RCCL]
    pack queries + pack target pyramid + build (all levels)      CorrBlock.__init__
    12 lookups with 12 different coordinate fields               12 x CorrBlock.__call__
value = 12 * (query voxels, all ranks) * steps / wall time (whole job).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Multi-GPU: the units are voxel-queries and they are independent.
Default --scaling weak: every rank owns its own volume pair (global batch = N),
so per-GPU work is fixed and there is no data-path collective (only the
timing barrier / max-reduce).  --scaling strong shards ONE pair's query voxels
by H slabs (ShardedCorrBlock: one RCCL all-gather of the fmap2 slabs per
forward), the north star's layout for 256^3 inputs (--size 64).

Prints one JSON line (rank 0) with roofline (dominant kernel, HIP-event timed
on its stream) and cpu_baseline (oracle/torch_cpu.py on the host, rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFS = 2500.0         # dense bf16 MFMA
F32_PEAK_TFS = 157.3           # f32 MFMA / vector


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=32, help="feature-map edge (32 = 128^3 input, 1/4 encoder)")
    ap.add_argument("--encoder", type=int, default=4, help="encoder downsampling (input edge = size x encoder)")
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--radius", type=int, default=4)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--impl", default="materialised", choices=["materialised", "fused"])
    ap.add_argument("--max-flow", type=float, default=2.0)
    ap.add_argument("--convc1", nargs="?", const="fused", default=None, choices=["fused", "unfused"],
                    help="each lookup also applies MotionEncoder.convc1 + ReLU: fused into the lookup "
                         "(dvc_corr_lookup_proj) or unfused (lookup, then torch conv3d + relu on the GPU)")
    ap.add_argument("--gather-output", action="store_true", help="strong scaling: all-gather every lookup output")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm); gloo only for rehearsals")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N>1: weak = one volume pair per rank (global batch N); strong = one pair's query "
                         "voxels sharded by H slabs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tune", default="", help="diagnostics: comma list key=value of dvc_set_tuning knobs")
    ap.add_argument("--cpu-rows", type=int, default=4096, help="query rows of the bounded CPU sample")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args()


def lookup_algorithmic_bytes(coords: torch.Tensor, dims, radius: int, store_bytes: int, out_bytes=None) -> float:
    """sum_q [ sum_l |W_l(q)| * store_bytes + 4 * L * (2r+1)^3 + 12 ].

    |W_l(q)| = prod_axes |[k - r, k + r + 1] intersect [0, S - 1]|, k = floor(coord / 2^l);
    levels with a size-1 axis read nothing."""
    L = len(dims)
    n3 = (2 * radius + 1) ** 3
    c = coords.reshape(coords.shape[0], 3, -1).double()
    nq = c.shape[0] * c.shape[2]
    win = torch.zeros((), dtype=torch.float64, device=c.device)
    for l, (H, W, D) in enumerate(dims):
        if min(H, W, D) == 1:
            continue
        tot = torch.ones_like(c[:, 0])
        for ax, S in enumerate((H, W, D)):
            k = torch.floor(c[:, ax] / 2 ** l)
            lo = torch.clamp(k - radius, min=0)
            hi = torch.clamp(k + radius + 1, max=S - 1)
            tot = tot * torch.clamp(hi - lo + 1, min=0)
        win = win + tot.sum()
    out_q = 4.0 * L * n3 if out_bytes is None else out_bytes   # --convc1: 96 fp32 per query instead
    return float(win.item()) * store_bytes + nq * (out_q + 12.0)


def cpu_baseline(args, f1, f2, coords_list):
    """oracle/torch_cpu.py (the reference op sequence) on a bounded row sample, host cores."""
    sys.path.insert(0, ROOT)
    from oracle import torch_cpu
    nthreads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(nthreads)
    f1c, f2c = f1.float().cpu(), f2.float().cpu()
    cc = [c.cpu() for c in coords_list]
    N = f1c[0, 0].numel()
    # the restatement materialises rows x N fp32 per level: cap it near 512 MB (128^3 fmaps: 64 rows)
    rows = min(args.cpu_rows, N, max(16, (1 << 27) // N))
    q0, q1 = 0, rows
    pyr = torch_cpu.build_rows(f1c, f2c, args.levels, q0, q1)           # warmup (allocations)
    torch_cpu.lookup_rows(pyr, cc[0], args.radius, False, q0, q1)
    t0 = time.perf_counter()
    pyr = torch_cpu.build_rows(f1c, f2c, args.levels, q0, q1)
    t_build = time.perf_counter() - t0
    nl = 3
    t0 = time.perf_counter()
    for i in range(nl):
        torch_cpu.lookup_rows(pyr, cc[i], args.radius, False, q0, q1)
    t_lookup = (time.perf_counter() - t0) / nl
    t_step = t_build + args.iters * t_lookup
    return {
        "value": args.iters * rows / t_step, "unit": "voxel-queries/s", "cores": nthreads, "kind": "port",
        "sample": (f"oracle/torch_cpu.py (reference op sequence, bit-identical to corr.py), fp32, query rows "
                   f"[0,{rows}) of {N}: build {t_build * 1e3:.0f} ms + {args.iters} x lookup "
                   f"{t_lookup * 1e3:.0f} ms (mean of {nl}); rows are independent, rate is per row"),
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if os.environ.get("DVCCORR_BENCH_ONE_DEVICE") == "1":   # rehearsal of N ranks on a 1-GPU box
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist
        if args.dist_backend == "nccl":
            tdist.init_process_group("nccl", device_id=dev)
        else:
            tdist.init_process_group(args.dist_backend)
    import dvccorr
    from dvccorr import ops
    from dvccorr import _lib
    from dvccorr.sharded import LOCAL, ShardedCorrBlock, slab_bounds
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.set_tuning(k, int(v))

    S, C, L, R = args.size, args.channels, args.levels, args.radius
    B = 1
    strong = args.scaling == "strong" and dist
    # weak scaling: each rank's own pair (seeded by rank); strong: every rank generates the same pair
    g = torch.Generator(device="cpu").manual_seed(1234 + (0 if strong else rank))
    f1 = torch.randn(B, C, S, S, S, generator=g)
    f2 = torch.randn(B, C, S, S, S, generator=g)
    base = dvccorr.coords_grid_3d(B, S, S, S, torch.device("cpu"))
    coords_list = [base + (torch.rand(B, 3, S, S, S, generator=g) * 2 - 1) * args.max_flow
                   for _ in range(args.iters)]
    h0, h1 = slab_bounds(S, world, rank) if strong else (0, S)
    f1_slab = f1[:, :, h0:h1].contiguous().to(dev)
    f2_slab = f2[:, :, h0:h1].contiguous().to(dev)
    coords_slab = [c[:, :, h0:h1].contiguous().to(dev) for c in coords_list]
    nq_local = (h1 - h0) * S * S
    nq_total = S * S * S * (1 if strong else world)   # query voxels of the whole job
    lay = dvccorr.layout(S, S, S, L, C)
    dims = lay.levels()
    store_bytes = 2 if args.precision == "bf16" else 4
    stream = torch.cuda.current_stream(dev)
    group = None

    ev = {"lookup": [], "build": []}
    proj_w = proj_b = None
    if args.convc1:   # random-init convc1 (Conv3d(L (2r+1)^3, 96, 1) default init range, update.py:222)
        K = L * (2 * R + 1) ** 3
        proj_w = ((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev)
        proj_b = ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev)

    def step(timed: bool):
        blk = ShardedCorrBlock(f1_slab, f2_slab, S, L, R, precision=args.precision, impl=args.impl,
                               group=group if strong else LOCAL, gather_output=args.gather_output,
                               build_events=ev["build"] if timed else None)
        for i in range(args.iters):
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            if args.convc1 == "fused":
                blk.lookup_convc1(coords_slab[i], proj_w, proj_b)
            elif args.convc1 == "unfused":
                torch.relu(torch.nn.functional.conv3d(blk(coords_slab[i]), proj_w.view(96, -1, 1, 1, 1), proj_b))
            else:
                blk(coords_slab[i])
            if timed:
                e1.record(stream)
                ev["lookup"].append((e0, e1))

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    with torch.no_grad():
        for _ in range(args.warmup):
            step(False)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(True)
        barrier()
        elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev if args.dist_backend == "nccl" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    lk_ms = [a.elapsed_time(b) for a, b in ev["lookup"]]
    bd_ms = [a.elapsed_time(b) for a, b in ev["build"]]
    lk_avg = sum(lk_ms) / max(len(lk_ms), 1)
    bd_avg = sum(bd_ms) / max(len(bd_ms), 1)
    ms_per_step = elapsed * 1e3 / args.steps
    value = args.iters * nq_total * args.steps / elapsed

    # roofline of the dominant kernel (by time per step, rank 0's view)
    lk_bytes = sum(lookup_algorithmic_bytes(c, dims, R, store_bytes if args.impl == "materialised" else 0,
                                            96 * 4.0 if args.convc1 == "fused" else None)
                   for c in coords_slab) / len(coords_slab)
    unpadded = sum(h * w * d for (h, w, d) in dims)
    n_targets = S * S * S
    if args.impl == "materialised":
        bd_bytes = nq_local * unpadded * store_bytes + 2 * C * 4 * n_targets
        bd_flops = 2.0 * nq_local * n_targets * C
    else:   # fused: the "build" only packs fmap1 rows and the pooled fmap2 pyramid (read f32, write bf16/f32)
        bd_bytes = (nq_local + n_targets) * C * 4 + (nq_local + unpadded) * C * store_bytes
        bd_flops = 0.0
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            tf = json.load(open(args.traffic_file))
            key = f"{args.impl}_{args.precision}_{S}_L{L}_r{R}_n{world if strong else 1}" + \
                (f"_convc1_{args.convc1}" if args.convc1 else "")
            traffic = tf.get(key, {}).get("lookup_hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if args.iters * lk_avg >= bd_avg or args.impl == "fused":
        achieved = lk_bytes / (lk_avg * 1e-3) / 1e9
        if args.impl == "materialised":
            kname = {"fused": "k_lookup_tile<PROJ> (dvc_corr_lookup_proj, convc1 fused)",
                     "unfused": "k_lookup_tile (dvc_corr_lookup) + torch conv3d/relu (timed together)"}.get(
                         args.convc1, "k_lookup_tile (dvc_corr_lookup)")
        elif args.precision == "bf16" and 1 <= R <= 4:
            kname = "k_fused_box (dvc_corr_lookup_fused)"
        else:
            kname = "k_fused_dots + k_lookup_win (dvc_corr_lookup_fused)"
        roof = {"kernel": kname,
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": lk_bytes, "avg_launch_ms": round(lk_avg, 4)}
        if args.impl == "fused":
            # the reference OTF dot count 2 C (2r+1)^3 L per voxel-query, against the dtype's MFMA peak
            fl = 2.0 * C * (2 * R + 1) ** 3 * L * nq_local
            peak = BF16_PEAK_TFS if args.precision == "bf16" else F32_PEAK_TFS
            roof["mfma"] = {"achieved": round(fl / (lk_avg * 1e-3) / 1e12, 1), "peak": peak, "unit": "TFLOP/s",
                            "frac": round(fl / (lk_avg * 1e-3) / 1e12 / peak, 4), "flops_per_launch": fl}
    else:
        achieved = bd_bytes / (bd_avg * 1e-3) / 1e9
        roof = {"kernel": "build (pack + k_build_bf16/f32)", "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "algorithmic_bytes_per_launch": bd_bytes, "avg_launch_ms": round(bd_avg, 4)}
    build_info = {"avg_ms": round(bd_avg, 4), "GB/s": round(bd_bytes / (bd_avg * 1e-3) / 1e9, 1) if bd_avg else None,
                  "TFLOP/s": round(bd_flops / (bd_avg * 1e-3) / 1e12, 1) if bd_avg and bd_flops else None}

    # per-iteration tail (raft_dvc.py:482-485), outside the timed region:
    # coords1 += delta_flow; flow_up = upflow_3d(coords1 - coords0) to the input size, one k_upflow pass
    tail = None
    with torch.no_grad():
        T = args.encoder * S
        c1 = coords_slab[0][:, :, :].reshape(B, 3, -1, S, S)
        dfl = (coords_slab[-1] - coords_slab[0]).reshape(c1.shape)
        h_lo = c1.shape[2]
        for _ in range(3):
            dvccorr.flow_step(c1, dfl, (h_lo * args.encoder, T, T))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        outs = [(torch.empty_like(c1), torch.empty((B, 3, h_lo * args.encoder, T, T), device=dev))
                for _ in range(2)]
        a.record(stream)
        for k in range(20):   # back-to-back on the stream (C ABI direct: no per-call allocation)
            n_, u_ = outs[k % 2]
            _lib.check(_lib.lib().dvc_flow_step(c1.data_ptr(), dfl.data_ptr(), n_.data_ptr(), u_.data_ptr(), B,
                                                h_lo, S, S, h_lo * args.encoder, T, T, stream.cuda_stream))
        b.record(stream)
        torch.cuda.synchronize()
        tail_ms = a.elapsed_time(b) / 20
        lo_b = 3 * 4 * c1[0, 0].numel() * B
        tail_bytes = 3 * lo_b + lo_b * args.encoder ** 3      # read coords1 + delta, write coords1; write flow_up
        tail = {"kernel": "k_upflow<DELTA,SUBGRID> (dvc_flow_step)", "avg_ms": round(tail_ms, 4),
                "algorithmic_bytes": tail_bytes,
                "GB/s": round(tail_bytes / (tail_ms * 1e-3) / 1e9, 1)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, f1, f2, coords_list)

    if rank == 0:
        line = {
            "metric": f"corr build+lookup voxel-queries/s ({args.encoder * S}^3 pair, 1/{args.encoder} encoder)",
            "value": value, "unit": "voxel-queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "bf16" if args.precision == "bf16" else "f32",
            "data": "synthetic: N(0,1) feature maps, coords = identity + U(-2,2), 12 coord fields per step",
            "config": {"workload": f"corr build + {args.iters} lookups{f' + convc1 ({args.convc1})' if args.convc1 else ''}, {S}^3 x {C} fmaps ({args.encoder * S}^3 "
                                   f"input, 1/{args.encoder} encoder), L={L}, r={R}, {args.impl}, {args.precision} build / fp32 lookup",
                       "global_batch": B if strong else B * world, "query_voxels": nq_total, "levels": L,
                       "radius": R,
                       "parallelism": (f"query-voxel H-slabs x{world}" if strong else
                                       f"one volume pair per rank x{world} (no data-path collective)") +
                                      (", output all-gather" if
                                                                          args.gather_output else "")},
            "roofline": roof,
            "build": build_info,
            "lookup_avg_ms": round(lk_avg, 4),
            "flow_step": tail,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
