#!/usr/bin/env python3
"""Benchmark of the RAFT-DVC correlation hot path on MI355X.

Metric (BASELINE.json): corr build+lookup voxel-queries/s, 128^3 pair, 1/4
encoder (32^3 x 128-channel feature maps), L=4, r=4, bf16-MFMA build, fp32
lookup, on 1/2/4/8 GPUs.  One step = one RAFTDVC forward's worth of
correlation work (corr.py:116-208 called as raft_dvc.py:414-450 calls it):
    [N>1: RCCL all-gather of the fmap2 H-slabs]                  fmap2 replication
    pack queries + pack target pyramid + build (all levels)      CorrBlock.__init__
    12 lookups with 12 different coordinate fields               12 x CorrBlock.__call__
value = 12 * (query voxels of the whole job) * steps / wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (what the driver runs)

`--gpus N` without a torchrun environment spawns torch.distributed.run with N
ranks as a child process (this parent never touches the GPU) and exits with
its code.

Multi-GPU, default --scaling strong: ONE volume pair's query
voxels are split into N H-slabs, one per rank; each rank all-gathers the fmap2
slabs (RCCL, the data-path collective), builds only its own rows of every
level and looks up its own queries; lookups stay shard-resident.  The per-rank
step after the collective is replayed as a HIP graph (--no-graph: eager).
At N>1 the line also carries `scaling_detail`, measured in the same job:
T1 (rank 0 alone on the whole problem), the strong layout with every lookup
all-gathered (--gather-output), weak scaling (one pair per rank) and config #4
(256^3 input, 1/4 encoder: 64^3 fmaps) strong-scaled, each with E(n) =
T1 / (n * Tn).

Prints one JSON line (rank 0) with roofline (dominant kernel, HIP-event timed
on its stream) and cpu_baseline (oracle/torch_cpu.py on the host, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-dvc_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFS = 2500.0         # dense bf16 MFMA
F32_PEAK_TFS = 157.3           # f32 MFMA / vector


def parse(argv=None):
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
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="pyramid / operand precision: bf16 (BASELINE config #3), fp16 (the reference Trainer's AMP), "
                         "fp32 (exact)")
    ap.add_argument("--impl", default="materialised", choices=["materialised", "fused"])
    ap.add_argument("--max-flow", type=float, default=2.0)
    ap.add_argument("--flow", default="random", choices=["random", "smooth"],
                    help="synthetic displacement field: random = i.i.d. U(-max_flow, max_flow) per voxel and axis "
                         "(default; the worst case for the union-of-windows fused kernels), smooth = a sum of "
                         "three low-frequency sinusoids per axis bounded by max_flow (a deformation field, as "
                         "RAFT-DVC's upsampled flow estimates are)")
    ap.add_argument("--convc1", nargs="?", const="fused", default=None, choices=["fused", "unfused"],
                    help="each lookup also applies MotionEncoder.convc1 + ReLU: fused into the lookup "
                         "(dvc_corr_lookup_proj) or unfused (lookup, then torch conv3d + relu on the GPU)")
    ap.add_argument("--gather-output", action="store_true", help="strong scaling: all-gather every lookup output")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm); gloo only with --rehearsal")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow a non-RCCL backend (gloo) for N>1: a rehearsal of the call sites on one device, "
                         "labelled as such; its numbers are not RCCL numbers")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="N>1: strong = one pair's query voxels sharded by H slabs (default); weak = one volume "
                         "pair per rank (global batch N)")
    ap.add_argument("--overlap", dest="overlap", action="store_true", default=False,
                    help="N>1 strong: overlap the next step's fmap2 all-gather with this step's compute in the "
                         "headline (default: the collective on the critical path; the overlapped figure is "
                         "reported in scaling_detail)")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="replay each rank's post-collective step as a HIP graph (default)")
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--no-extras", action="store_true", help="N>1: skip scaling_detail (T1, gather, weak, cfg #4)")
    ap.add_argument("--cfg4-steps", type=int, default=3, help="N>1: timed steps of the config #4 extra (0: off)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="diagnostics on one GPU: time rank --shard-rank's slab of an N-way split alone "
                         "(its per-rank compute; fmap2 is given whole, no collective)")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tune", default="", help="diagnostics: comma list key=value of dvc_set_tuning knobs")
    ap.add_argument("--cpu-rows", type=int, default=4096, help="query rows of the bounded CPU sample")
    ap.add_argument("--coord-fields", type=int, default=0,
                    help="diagnostics: distinct coordinate fields the step's lookups cycle through (0 = one per lookup, "
                         "the metric's setting; 1 = every lookup at the same coordinates: the reuse bound)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args(argv)


def spawn(args) -> int:
    """`bench.py --gpus N` outside torchrun: launch N ranks with torch.distributed.run as a child process."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: spawning {args.gpus} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


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


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the job's CPU share where the environment states it
    (OMP_NUM_THREADS on the GPU box), else every CPU the process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(args, f1, f2, coords_list):
    """oracle/torch_cpu.py (the reference op sequence) on a bounded row sample, host cores; min of 3 runs."""
    sys.path.insert(0, ROOT)
    from oracle import torch_cpu
    nthreads = cpu_threads()
    torch.set_num_threads(nthreads)
    f1c, f2c = f1.float().cpu(), f2.float().cpu()
    cc = [c.cpu() for c in coords_list]
    N = f1c[0, 0].numel()
    # the restatement materialises rows x N fp32 per level: cap it near 512 MB (128^3 fmaps: 64 rows)
    rows = min(args.cpu_rows, N, max(16, (1 << 27) // N))
    q0, q1 = 0, rows
    pyr = torch_cpu.build_rows(f1c, f2c, args.levels, q0, q1)           # warmup (allocations)
    torch_cpu.lookup_rows(pyr, cc[0], args.radius, False, q0, q1)
    tb, tl = [], []
    for i in range(3):
        t0 = time.perf_counter()
        pyr = torch_cpu.build_rows(f1c, f2c, args.levels, q0, q1)
        tb.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        torch_cpu.lookup_rows(pyr, cc[i], args.radius, False, q0, q1)
        tl.append(time.perf_counter() - t0)
    t_build, t_lookup = min(tb), min(tl)
    t_step = t_build + args.iters * t_lookup
    return {
        "value": args.iters * rows / t_step, "unit": "voxel-queries/s", "cores": nthreads, "kind": "port",
        "host_cpus": os.cpu_count(),
        "sample": (f"oracle/torch_cpu.py (reference op sequence, bit-identical to corr.py), fp32, {nthreads} "
                   f"threads, query rows [0,{rows}) of {N}: build {t_build * 1e3:.0f} ms + {args.iters} x lookup "
                   f"{t_lookup * 1e3:.0f} ms (min of 3 runs); rows are independent, rate is per row"),
    }


class Runner:
    """One rank's correlation step: [all-gather of the fmap2 slabs] + pack/build + `iters` lookups.

    The collective is issued eagerly; everything after it is optionally captured once as a HIP graph
    (torch.cuda.CUDAGraph over the stream-ordered, allocation-free C ABI) and replayed, which removes the
    host launch cost of the 15 launches per step when the per-rank work is small.

    overlap=True (sharded runs): the fmap2 all-gather of step k+1 is issued asynchronously (RCCL's own
    stream) while step k computes, into the other half of a double-buffered receive buffer -- consecutive
    forwards pipelined the way a serving loop would run them.  Every step still gathers, builds and looks
    up in full; only the collective's latency is hidden behind the previous step's lookups."""

    def __init__(self, f1_slab, f2_slab, coords_slabs, H, args, group, world, gather_output=False,
                 graph=True, proj=None, overlap=False):
        from dvccorr.sharded import LOCAL
        self.args, self.group, self.H = args, group, H
        self.world = 1 if group == LOCAL else world
        self.gather_output = gather_output and self.world > 1
        B, C = f1_slab.shape[:2]
        self.f1_flat = f1_slab.reshape(B, C, -1).contiguous()
        self.f2_slab = f2_slab.contiguous()
        self.coords = [c.reshape(B, 3, -1).contiguous() for c in coords_slabs]
        self.slab_shape = tuple(f1_slab.shape)
        self.proj = proj
        self.bufs = [None, None]
        self.overlap = overlap and self.world > 1 and not self.gather_output
        if self.world > 1:
            from dvccorr.sharded import all_gather_slab
            # the static receive buffer(s) (two when the next step's gather overlaps this step's compute)
            self.bufs = [all_gather_slab(self.f2_slab, H, group) for _ in range(2 if self.overlap else 1)]
        self.use_graph = graph and not self.gather_output
        self.graphs = [None, None]
        self.outs = None
        self.k = 0            # step counter (selects the receive buffer)
        self.pending = None   # async work handle of the next step's gather

    def collective(self, slot=0, async_op=False):
        if self.world > 1:
            from dvccorr.sharded import all_gather_slab
            if async_op:
                return all_gather_slab(self.f2_slab, self.H, self.group, buf=self.bufs[slot], async_op=True)
            all_gather_slab(self.f2_slab, self.H, self.group, buf=self.bufs[slot])
        return None

    def compute(self, ev=None, stream=None, slot=0):
        from dvccorr.sharded import HipRows, gather_slabs
        a = self.args
        if ev is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        if self.world > 1:   # the targets packed straight from the all-gather's receive buffer (no assembled fmap2)
            rows = HipRows(self.f1_flat, None, a.levels, a.radius, False, a.precision, a.impl,
                           gathered=(self.bufs[slot], self.H))
        else:
            rows = HipRows(self.f1_flat, self.f2_slab, a.levels, a.radius, False, a.precision, a.impl)
        if ev is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(stream)
            ev["build"].append((e0, e1))
        outs = []
        for c in self.coords:
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            if a.convc1 == "fused":
                o = rows.lookup_convc1(c, *self.proj)
            elif a.convc1 == "unfused":
                o = rows.lookup(c)
                o = torch.relu(torch.nn.functional.conv1d(o, self.proj[0].view(96, -1, 1), self.proj[1]))
            else:
                o = rows.lookup(c)
            if ev is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(stream)
                ev["lookup"].append((e0, e1))
            if self.gather_output:
                B = o.shape[0]
                o = gather_slabs(o.view(B, o.shape[1], -1, *self.slab_shape[3:]), self.H, self.group)
            outs.append(o)
        return outs

    def capture(self, slot):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.compute(slot=slot)                # warm-up outside the capture (library load, attributes)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.outs = self.compute(slot=slot)
        self.graphs[slot] = g

    def _run(self, slot):
        if self.use_graph:
            if self.graphs[slot] is None:
                self.capture(slot)
            self.graphs[slot].replay()
        else:
            self.outs = self.compute(slot=slot)

    def step(self):
        if not self.overlap:
            self.collective()
            self._run(0)
            return
        slot = self.k & 1
        if self.pending is None:                   # first step: nothing in flight yet
            self.pending = self.collective(slot, async_op=True)
        self.pending.wait()                        # this step's fmap2 is in bufs[slot]
        # the next step's gather goes into the other buffer, which the previous step's compute (already
        # enqueued before this point) has finished reading by the time RCCL's stream starts it
        self.pending = self.collective(slot ^ 1, async_op=True)
        self._run(slot)
        self.k += 1

    def drain(self):
        if self.pending is not None:
            self.pending.wait()
            self.pending = None

    def release(self):
        self.drain()
        self.graphs = [None, None]
        self.outs = None
        self.bufs = [None, None]


def timed(runner, steps, warmup, dist, dev, participate=True):
    """warmup untimed steps, then `steps` timed ones bracketed by barrier + synchronize; max over ranks."""
    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    with torch.no_grad():
        if participate:
            for _ in range(warmup):
                runner.step()
            runner.drain()
        barrier()
        t0 = time.perf_counter()
        if participate:
            for _ in range(steps):
                runner.step()
            runner.drain()
        barrier()
        elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev if torch.distributed.get_backend() == "nccl" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def synthetic_flow(kind, B, S, max_flow, g):
    """(B, 3, S, S, S) displacement: i.i.d. uniform, or per axis a sum of three sinusoids
    (max_flow / 3) sin(2 pi k.p / S + phase) with random integer wave vectors k in [0, 2]^3."""
    if kind == "random":
        return (torch.rand(B, 3, S, S, S, generator=g) * 2 - 1) * max_flow
    ax = torch.arange(S, dtype=torch.float32)
    p = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"))           # (3, S, S, S)
    out = torch.zeros(B, 3, S, S, S)
    for bb in range(B):
        for c in range(3):
            for _ in range(3):
                k = torch.randint(0, 3, (3,), generator=g).float()
                ph = float(torch.rand((), generator=g)) * 2 * torch.pi
                out[bb, c] += (max_flow / 3) * torch.sin(2 * torch.pi * (k[:, None, None, None] * p).sum(0) / S + ph)
    return out


def gpu_inputs(S, C, iters, max_flow, seed, dev):
    """Seeded inputs generated on the GPU (identical on every rank of one node)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    f1 = torch.randn(1, C, S, S, S, device=dev, generator=g)
    f2 = torch.randn(1, C, S, S, S, device=dev, generator=g)
    ax = torch.arange(S, device=dev, dtype=torch.float32)
    base = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"))[None]
    coords = [base + (torch.rand(1, 3, S, S, S, device=dev, generator=g) * 2 - 1) * max_flow for _ in range(iters)]
    return f1, f2, coords


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = world > 1
    if dist and args.dist_backend != "nccl" and not args.rehearsal:
        raise SystemExit(f"bench.py: --dist-backend {args.dist_backend} is a rehearsal backend; pass --rehearsal "
                         f"to run it (the line is then labelled as a rehearsal, not RCCL)")
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
        assert tdist.get_world_size() == args.gpus, (tdist.get_world_size(), args.gpus)
    import dvccorr
    from dvccorr import _lib
    from dvccorr.sharded import LOCAL, slab_bounds
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.set_tuning(k, int(v))

    S, C, L, R = args.size, args.channels, args.levels, args.radius
    B = 1
    strong = args.scaling == "strong"
    shard_diag = args.shard_of > 1 and not dist
    # strong: every rank generates the same pair; weak: each rank its own (seeded by rank)
    g = torch.Generator(device="cpu").manual_seed(1234 + (0 if strong else rank))
    f1 = torch.randn(B, C, S, S, S, generator=g)
    f2 = torch.randn(B, C, S, S, S, generator=g)
    base = dvccorr.coords_grid_3d(B, S, S, S, torch.device("cpu"))
    nfields = args.iters if args.coord_fields <= 0 else min(args.coord_fields, args.iters)
    fields = [base + synthetic_flow(args.flow, B, S, args.max_flow, g) for _ in range(nfields)]
    coords_list = [fields[i % nfields] for i in range(args.iters)]
    if shard_diag:
        h0, h1 = slab_bounds(S, args.shard_of, args.shard_rank)
    else:
        h0, h1 = slab_bounds(S, world, rank) if (strong and dist) else (0, S)
    f1_slab = f1[:, :, h0:h1].contiguous().to(dev)
    f2_slab = (f2 if shard_diag else f2[:, :, h0:h1]).contiguous().to(dev)
    coords_slab = [c[:, :, h0:h1].contiguous().to(dev) for c in coords_list]
    nq_local = (h1 - h0) * S * S
    nq_total = S * S * S * (1 if strong else world) if not shard_diag else nq_local
    lay = dvccorr.layout(S, S, S, L, C)
    dims = lay.levels()
    sixteen = args.precision in ("bf16", "fp16")
    store_bytes = 2 if sixteen else 4
    stream = torch.cuda.current_stream(dev)
    group = None if (strong and dist) else LOCAL

    proj = None
    if args.convc1:   # random-init convc1 (Conv3d(L (2r+1)^3, 96, 1) default init range, update.py:222)
        K = L * (2 * R + 1) ** 3
        proj = (((torch.rand(96, K, generator=g) * 2 - 1) / K ** 0.5).to(dev),
                ((torch.rand(96, generator=g) * 2 - 1) / K ** 0.5).to(dev))

    runner = Runner(f1_slab, f2_slab, coords_slab, S, args, group, world, gather_output=args.gather_output,
                    graph=args.graph, proj=proj, overlap=args.overlap)
    elapsed = timed(runner, args.steps, args.warmup, dist, dev)
    runner.release()
    ms_per_step = elapsed * 1e3 / args.steps
    value = args.iters * nq_total * args.steps / elapsed

    # per-kernel HIP-event timing on the launch stream: eager steps after the timed region
    ev = {"lookup": [], "build": []}
    with torch.no_grad():
        er = Runner(f1_slab, f2_slab, coords_slab, S, args, group, world, graph=False, proj=proj)
        for k in range(4):
            er.collective()
            er.compute(ev if k > 0 else None, stream)
        torch.cuda.synchronize()
        er.release()
        del er
    lk_ms = [a.elapsed_time(b) for a, b in ev["lookup"]]
    bd_ms = [a.elapsed_time(b) for a, b in ev["build"]]
    lk_avg = sum(lk_ms) / max(len(lk_ms), 1)
    bd_avg = sum(bd_ms) / max(len(bd_ms), 1)

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
    traffic = traffic_src = None
    if os.path.exists(args.traffic_file) and not shard_diag and args.flow == "random":   # PMC passes are per workload
        try:
            tf = json.load(open(args.traffic_file))
            key = f"{args.impl}_{args.precision}_{S}_L{L}_r{R}_n{world if strong else 1}" + \
                (f"_convc1_{args.convc1}" if args.convc1 else "")
            traffic = tf.get(key, {}).get("lookup_hbm_bytes_per_launch")
            traffic_src = tf.get(key, {}).get("note") if traffic is not None else None
        except Exception:
            traffic = None
    lk_roof = lk_bytes / (lk_avg * 1e-3) / 1e9 if lk_avg else 0.0
    if args.iters * lk_avg >= bd_avg or args.impl == "fused":
        achieved = lk_roof
        if args.impl == "materialised":
            kname = {"fused": "k_lookup_tile<PROJ> (dvc_corr_lookup_proj, convc1 fused)",
                     "unfused": "k_lookup_tile (dvc_corr_lookup) + torch conv/relu (timed together)"}.get(
                         args.convc1, "k_lookup_tile (dvc_corr_lookup)")
        elif args.convc1 == "fused" and sixteen and 1 <= R <= 4:
            kname = ("k_otf_keys + radix sort + k_fused_proj + k_rows_to_channels "
                     "(dvc_corr_lookup_fused_proj, convc1 fused, timed together)")
        elif sixteen and 1 <= R <= 4:
            kname = "k_fused_box (dvc_corr_lookup_fused)"
        elif 1 <= R <= 4 and "fused_variant=0" not in args.tune:
            kname = "k_fused_box_f32 (dvc_corr_lookup_fused; fp32 operands as three bf16 pieces, six MFMAs per step)"
        else:
            kname = "k_fused_dots + k_lookup_win (dvc_corr_lookup_fused)"
        roof = {"kernel": kname,
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": lk_bytes, "avg_launch_ms": round(lk_avg, 4),
                "traffic_source": traffic_src}   # which PMC pass (file, tree) the traffic figure comes from
        if args.impl == "fused":
            # the reference OTF dot count 2 C (2r+1)^3 L per voxel-query, against the dtype's MFMA peak
            fl = 2.0 * C * (2 * R + 1) ** 3 * L * nq_local
            peak = BF16_PEAK_TFS if sixteen else F32_PEAK_TFS   # (fp16 MFMA: the bf16 rate)
            if args.convc1 == "fused":   # + convc1: 2 x 96 x L (2r+1)^3 per voxel-query
                fl += 2.0 * 96 * (2 * R + 1) ** 3 * L * nq_local
            roof["mfma"] = {"achieved": round(fl / (lk_avg * 1e-3) / 1e12, 1), "peak": peak, "unit": "TFLOP/s",
                            "frac": round(fl / (lk_avg * 1e-3) / 1e12 / peak, 4), "flops_per_launch": fl}
            if args.convc1 == "fused":
                # nothing per lookup channel reaches HBM (96 fp32 per query out): the bound is the matrix
                # cores, so the top-level roofline is the MFMA one and the HBM numbers move to a sub-block
                hbm = {k: roof[k] for k in ("achieved", "peak", "unit", "frac", "traffic")}
                roof.update({"bound": "mfma", "achieved": roof["mfma"]["achieved"], "peak": peak,
                             "unit": "TFLOP/s", "frac": roof["mfma"]["frac"], "traffic": None, "hbm": hbm})
    else:
        # the bf16 build (C = 128) is HBM-write-bound (~112 FLOP/B < ridge ~312); the exact-f32
        # build is bound by the f32 matrix cores (~56 FLOP/B > ridge ~20): report each against its own roof
        gbs = bd_bytes / (bd_avg * 1e-3) / 1e9
        tfs = bd_flops / (bd_avg * 1e-3) / 1e12
        lk = {"achieved": round(lk_roof, 1), "frac": round(lk_roof / HBM_PEAK_GBS, 4),
              "algorithmic_bytes_per_launch": lk_bytes, "avg_launch_ms": round(lk_avg, 4)}
        if args.precision == "fp32":
            roof = {"kernel": "build (pack + k_build_f32r, exact-f32 MFMA v_mfma_f32_32x32x2_f32, register-resident "
                              "targets)", "bound": "mfma",
                    "achieved": round(tfs, 1), "peak": F32_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": round(tfs / F32_PEAK_TFS, 4), "traffic": None, "flops_per_launch": bd_flops,
                    "avg_launch_ms": round(bd_avg, 4),
                    "hbm": {"achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                            "algorithmic_bytes_per_launch": bd_bytes},
                    "lookup": lk}
        else:
            roof = {"kernel": f"build (pack + k_build_bf16_2b, {args.precision})", "bound": "hbm", "achieved": round(gbs, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                    "algorithmic_bytes_per_launch": bd_bytes, "avg_launch_ms": round(bd_avg, 4),
                    "mfma": {"achieved": round(tfs, 1), "peak": BF16_PEAK_TFS,
                             "frac": round(tfs / BF16_PEAK_TFS, 4), "flops_per_launch": bd_flops},
                    "lookup": lk}
    build_info = {"avg_ms": round(bd_avg, 4), "GB/s": round(bd_bytes / (bd_avg * 1e-3) / 1e9, 1) if bd_avg else None,
                  "TFLOP/s": round(bd_flops / (bd_avg * 1e-3) / 1e12, 1) if bd_avg and bd_flops else None}
    if bd_avg and bd_flops:   # each build against its binding roof
        build_info["roof"] = ("f32 mfma" if args.precision == "fp32" else "hbm write")
        build_info["frac"] = round(bd_flops / (bd_avg * 1e-3) / 1e12 / F32_PEAK_TFS, 4) if args.precision == "fp32" \
            else round(bd_bytes / (bd_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    if rank == 0 and world == 1 and not shard_diag and roof.get("bound") == "hbm" and roof.get("unit") == "GB/s":
        # context for the HBM fraction: the plain device copy rate of this box (read + write bytes), and the
        # kernel's counter traffic per launch at its measured time, against it (traffic from the PMC file above)
        cp = copy_rate(dev, stream)
        roof["same_box_copy"] = cp
        if roof.get("traffic"):
            tr = roof["traffic"] / (roof["avg_launch_ms"] * 1e-3) / 1e9
            roof["traffic_gbs"] = round(tr, 1)
            roof["traffic_frac_of_copy"] = round(tr / cp["GB/s"], 3)
    tail = flow_tail(args, coords_slab, S, B, dev, stream, _lib, dvccorr)
    bwd = bwd_amp = None
    if world == 1 and not shard_diag and args.convc1 is None:
        bwd = backward_timing(args, f1_slab, f2_slab, coords_slab, dims, dev, stream)
        # the reference Trainer's AMP backward (fp16 pyramid, trainer.py:249-257) on the same inputs
        bwd_amp = backward_timing(args, f1_slab, f2_slab, coords_slab, dims, dev, stream, "fp16")

    detail = None
    if dist and strong and not args.no_extras:
        detail = scaling_detail(args, f1, f2, coords_list, ms_per_step, world, rank, dev, dist, group, proj)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not shard_diag:
        cpu = cpu_baseline(args, f1, f2, coords_list)

    if rank == 0:
        coll = "RCCL" if args.dist_backend == "nccl" else f"{args.dist_backend} (REHEARSAL, not RCCL)"
        par = (f"query-voxel H-slabs x{world}, {coll} all-gather of fmap2 per step" if (strong and dist) else
               f"one volume pair per rank x{world} (no data-path collective)" if dist else "single GPU")
        if shard_diag:
            par = f"diagnostic: rank {args.shard_rank}'s slab of a {args.shard_of}-way split alone (no collective)"
        line = {
            "metric": f"corr build+lookup voxel-queries/s ({args.encoder * S}^3 pair, 1/{args.encoder} encoder)",
            "value": value, "unit": "voxel-queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": {"bf16": "bf16", "fp16": "f16"}.get(args.precision, "f32"),
            "data": (f"synthetic: N(0,1) feature maps, coords = identity + "
                     + (f"U(-{args.max_flow:g},{args.max_flow:g}) i.i.d. per voxel" if args.flow == "random" else
                        f"a smooth field (3 sinusoids per axis, |flow| <= {args.max_flow:g})")
                     + f", {args.iters if args.coord_fields <= 0 else min(args.coord_fields, args.iters)} coord fields per step"),
            "config": {"workload": f"corr build + {args.iters} lookups{f' + convc1 ({args.convc1})' if args.convc1 else ''}, {S}^3 x {C} fmaps ({args.encoder * S}^3 "
                                   f"input, 1/{args.encoder} encoder), L={L}, r={R}, {args.impl}, {args.precision} build / fp32 lookup",
                       "global_batch": B if strong else B * world, "query_voxels": nq_total, "levels": L,
                       "radius": R, "parallelism": par + (", output all-gather" if args.gather_output else ""),
                       "step_replay": "hip graph after the collective" if runner.use_graph else "eager",
                       "collective": ("next step's fmap2 all-gather overlapped with this step's compute"
                                      if runner.overlap else "fmap2 all-gather before the step's compute"
                                      if runner.world > 1 else None)},
            "roofline": roof,
            "build": build_info,
            "lookup_avg_ms": round(lk_avg, 4),
            "flow_step": tail,
            "backward": bwd,
            "backward_amp": bwd_amp,
            "cpu_baseline": cpu,
        }
        if detail is not None:
            line["scaling_detail"] = detail
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


def copy_rate(dev, stream, nbytes=1 << 30, reps=7):
    """Device-to-device copy of 1 GiB (torch copy_, ROCm's own copy kernel): median read + write bytes per second.
    The mixed read/write rate a streaming kernel gets on this box, next to the 8 TB/s spec the fraction uses."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    b.copy_(a)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        b.copy_(a)
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    med = ts[len(ts) // 2]
    del a, b
    return {"GB/s": round(2 * nbytes / (med * 1e-3) / 1e9, 1), "what": "torch copy_ of 1 GiB, read + write bytes, "
            f"median of {reps}", "ms": round(med, 4)}


def backward_timing(args, f1, f2, coords, dims, dev, stream, precision=None):
    """The training path's backward (dvc_corr_backward: d fmap1, d fmap2 of one lookup; autograd through
    corr.py:141-208), HIP-event timed outside the timed region on the bench's inputs and a random output
    gradient, for the pyramid precision `precision` (default: the bench's; "fp16" = the reference Trainer's AMP
    pyramid, trainer.py:249-257).  Algorithmic bytes: read grad_out (fp32) + coords + the packed query/target
    rows, write d fmap1 + d fmap2 (fp32); FLOPs: 2 x 2 C per window dot (d fmap1 and d fmap2), (2r+2)^3 window
    dots per query and level."""
    from dvccorr import ops, _lib
    precision = precision or args.precision
    with torch.no_grad():
        B, C = f1.shape[:2]
        S = args.size
        L, R = args.levels, args.radius
        Nq = f1[0, 0].numel()
        dt = ops.dtype_code(precision)
        q = ops.pack_queries(f1.reshape(B, C, -1), dt)
        t = ops.pack_targets(f2, L, dt)
        g = torch.Generator(device=dev).manual_seed(99)
        gout = torch.randn(B, L * (2 * R + 1) ** 3, Nq, device=dev, generator=g)
        cf = coords[0].reshape(B, 3, -1).contiguous()
        for _ in range(2):
            ops.corr_backward(q, t, cf, gout, C, S, S, S, L, R, False, dt)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 5
        a.record(stream)
        for _ in range(n):
            ops.corr_backward(q, t, cf, gout, C, S, S, S, L, R, False, dt)
        b.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / n
    esz = 4 if precision == "fp32" else 2
    nbytes = gout.numel() * 4 + cf.numel() * 4 + (q.numel() + t.numel()) * esz + 2 * B * C * Nq * 4
    flops = 2.0 * 2 * C * (2 * R + 2) ** 3 * L * B * Nq
    mfma = bool(_lib.lib().dvc_corr_backward_mfma(B, Nq, C, S, S, S, L, R, 0, dt))
    gt = "k_grad_t_dense"
    kern = (f"k_win_grad + k_grad_q_mfma + counting sort + {gt} + k_unpack_sum (dvc_corr_backward, {precision} "
            f"operands on v_mfma_f32_32x32x16_{'f16' if precision == 'fp16' else 'bf16'})" if mfma else
            f"k_win_grad + k_grad_q + counting sort + k_grad_t + k_unpack_sum (dvc_corr_backward, {precision} operands, "
            f"fp32 VALU)")
    peak = F32_PEAK_TFS if precision == "fp32" else BF16_PEAK_TFS
    return {"precision": precision, "kernels": kern,
            "avg_ms": round(ms, 4), "algorithmic_bytes": nbytes, "GB/s": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "hbm_frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "flops": flops,
            "TFLOP/s": round(flops / (ms * 1e-3) / 1e12, 2),
            ("mfma_frac" if mfma else "valu_frac"): round(flops / (ms * 1e-3) / 1e12 / peak, 4)}


def flow_tail(args, coords_slab, S, B, dev, stream, _lib, dvccorr):
    """Per-iteration tail (raft_dvc.py:482-485), outside the timed region:
    coords1 += delta_flow; flow_up = upflow_3d(coords1 - coords0) to the input size, one k_upflow pass."""
    with torch.no_grad():
        T = args.encoder * S
        c1 = coords_slab[0].reshape(B, 3, -1, S, S)
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
        return {"kernel": "k_upflow<DELTA,SUBGRID> (dvc_flow_step)", "avg_ms": round(tail_ms, 4),
                "algorithmic_bytes": tail_bytes, "GB/s": round(tail_bytes / (tail_ms * 1e-3) / 1e9, 1)}


def scaling_detail(args, f1, f2, coords_list, ms_strong, world, rank, dev, dist, group, proj):
    """N>1, measured in the same job: T1 (rank 0 alone, whole problem), strong with the output all-gather,
    weak (one pair per rank) and config #4 (64^3 fmaps) strong-scaled; E(n) = T1 / (n Tn)."""
    from dvccorr.sharded import LOCAL, slab_bounds
    S = args.size
    steps, warm = args.steps, max(1, args.warmup)
    out = {"note": "E = T1 / (n * Tn); T1 = rank 0 alone on the whole problem, same job, same kernels"}
    # T1: rank 0 runs the unsharded step, the other ranks wait at the barriers
    full = [c.to(dev) for c in coords_list] if rank == 0 else None
    r1 = Runner(f1.to(dev), f2.to(dev), full, S, args, LOCAL, world, graph=args.graph, proj=proj) \
        if rank == 0 else None
    t1 = timed(r1, steps, warm, dist, dev, participate=rank == 0) * 1e3 / steps
    if r1 is not None:
        r1.release()
    del r1
    torch.cuda.empty_cache()
    out["cfg3_t1_ms"] = round(t1, 4)
    out["cfg3_strong_resident"] = {"ms_per_step": round(ms_strong, 4), "E": round(t1 / (world * ms_strong), 4)}
    # the same layout with the other collective placement than the headline's: serial (collective on the
    # critical path, the headline default) <-> overlapped (next step's all-gather under this step's compute)
    h0, h1 = slab_bounds(S, world, rank)
    rs = Runner(f1[:, :, h0:h1].contiguous().to(dev), f2[:, :, h0:h1].contiguous().to(dev),
                [c[:, :, h0:h1].contiguous().to(dev) for c in coords_list], S, args, group, world,
                graph=args.graph, proj=proj, overlap=not args.overlap)
    ts = timed(rs, steps, warm, dist, dev) * 1e3 / steps
    rs.release()
    key = "cfg3_strong_resident_serial_collective" if args.overlap else "cfg3_strong_resident_overlapped_collective"
    out[key] = {"ms_per_step": round(ts, 4), "E": round(t1 / (world * ts), 4)}
    h0, h1 = slab_bounds(S, world, rank)
    f1s, f2s = f1[:, :, h0:h1].contiguous().to(dev), f2[:, :, h0:h1].contiguous().to(dev)
    cs = [c[:, :, h0:h1].contiguous().to(dev) for c in coords_list]
    rg = Runner(f1s, f2s, cs, S, args, group, world, gather_output=True, graph=False, proj=proj)
    tg = timed(rg, steps, warm, dist, dev) * 1e3 / steps
    rg.release()
    out["cfg3_strong_gather_output"] = {"ms_per_step": round(tg, 4), "E": round(t1 / (world * tg), 4)}
    # weak: every rank its own whole pair (the same pair here; no collective)
    rw = Runner(f1.to(dev), f2.to(dev), [c.to(dev) for c in coords_list], S, args, LOCAL, world, graph=args.graph,
                proj=proj)
    tw = timed(rw, steps, warm, dist, dev) * 1e3 / steps
    rw.release()
    del rw
    torch.cuda.empty_cache()
    out["cfg3_weak"] = {"ms_per_step": round(tw, 4), "E": round(t1 / tw, 4),
                        "value": round(args.iters * S ** 3 * world / (tw * 1e-3), 1)}
    if args.cfg4_steps > 0 and args.impl == "materialised" and args.convc1 is None:
        out["cfg4"] = cfg4_strong(args, world, rank, dev, dist, group)
    return out


def cfg4_strong(args, world, rank, dev, dist, group):
    """Config #4 (256^3 input, 1/4 encoder: 64^3 x 128 fmaps, L=4, r=4, bf16): T1 on rank 0 alone (157 GB
    pyramid) and the H-slab layout on every rank (157/n GB each)."""
    from dvccorr.sharded import LOCAL, slab_bounds
    S, steps = 64, args.cfg4_steps
    a4 = parse([f"--size={S}", f"--channels={args.channels}", f"--levels={args.levels}", f"--radius={args.radius}",
                f"--iters={args.iters}", f"--precision={args.precision}"])
    f1, f2, coords = gpu_inputs(S, args.channels, args.iters, args.max_flow, 4004, dev)
    r1 = Runner(f1, f2, coords, S, a4, LOCAL, world, graph=False) if rank == 0 else None
    t1 = timed(r1, steps, 1, dist, dev, participate=rank == 0) * 1e3 / steps
    if r1 is not None:
        r1.release()
    del r1
    torch.cuda.empty_cache()
    h0, h1 = slab_bounds(S, world, rank)
    rn = Runner(f1[:, :, h0:h1].contiguous(), f2[:, :, h0:h1].contiguous(),
                [c[:, :, h0:h1].contiguous() for c in coords], S, a4, group, world, graph=args.graph,
                overlap=args.overlap)
    tn = timed(rn, steps, 1, dist, dev) * 1e3 / steps
    rn.release()
    del rn
    torch.cuda.empty_cache()
    return {"workload": "64^3 x 128 fmaps (256^3 input, 1/4 encoder), L=4, r=4, bf16, build + 12 lookups",
            "t1_ms": round(t1, 3), "tn_ms": round(tn, 3), "E": round(t1 / (world * tn), 4),
            "value": round(args.iters * S ** 3 / (tn * 1e-3), 1), "steps": steps}


if __name__ == "__main__":
    main()
