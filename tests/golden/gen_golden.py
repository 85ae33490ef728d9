#!/usr/bin/env python3
"""Generate the golden vectors by importing the reference -- survey container only.

    python tests/golden/gen_golden.py [--reference /root/reference]

The reference (zachtong/RAFT-DVC) is imported from its read-only checkout
and run on CPU; only its OUTPUTS (plus the seeds/shapes of the inputs, which
tests/prng.py regenerates bit-identically anywhere) are written here, as
small .npz files.  Nothing from the reference's source is stored.

Each fixture mirrors a reference test or a BASELINE configuration:
  sampler_kat.npz   tests/test_corr_sampler.py:33-71  (impulse, weights, legacy swap, random)
  peak_shift.npz    tests/test_corr_sampler.py:74-105 (CorrBlock peak location, both conventions)
  equiv_*.npz       tests/test_corr_equivalence.py:136-153 (B=2, C=16, 8^3, L in {1,2,4}, r in {3,4})
  edge_*.npz        non-cubic / size-1-level cases
  cfg2.npz, cfg3.npz BASELINE configs #2 (16^3) and #3 (32^3), C=128, L=4, r=4 (sampled rows + checksums)
  plumbing.npz      config #1: RAFTDVC 64^3, 1/8 encoder, L=4, 12 iters, random init (seeded):
                    the fmaps and per-iteration coords fed to CorrBlock, and its sampled outputs
It also checks oracle/torch_cpu.py bit-for-bit and oracle/corr_oracle.c to
tolerance against the reference, recording the result in golden_meta.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)

import prng  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from oracle import torch_cpu  # noqa: E402


def checksums(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float64)
    return np.array([x.sum(), np.abs(x).sum(), (x * x).sum(), np.abs(x).max()], np.float64)


def sample_rows(rng_seed: int, total: int, k: int) -> np.ndarray:
    u = prng.uniform24(rng_seed, 4 * k)
    rows = np.unique((u * total).astype(np.int64))[:k]
    return np.sort(rows)


def rows_of(out: np.ndarray, rows: np.ndarray) -> np.ndarray:
    """out (B, Ch, H, W, D) -> [len(rows), Ch] for global rows b*N + q."""
    B, Ch = out.shape[:2]
    flat = out.reshape(B, Ch, -1)
    N = flat.shape[2]
    return np.stack([flat[r // N, :, r % N] for r in rows]).astype(np.float32)


class Gen:
    def __init__(self, ref_root: str):
        sys.path.insert(0, ref_root)
        from src.core.corr import CorrBlock, bilinear_sampler_3d  # type: ignore
        self.CorrBlock = CorrBlock
        self.sampler = bilinear_sampler_3d
        self.meta = {"torch": torch.__version__, "numpy": np.__version__, "threads": torch.get_num_threads(),
                     "reference": "zachtong/RAFT-DVC @ /root/reference (read-only)", "fixtures": {},
                     "oracle_checks": []}

    def save(self, name: str, **arrays):
        path = os.path.join(HERE, name)
        np.savez_compressed(path, **arrays)
        self.meta["fixtures"][name] = {k: list(np.shape(v)) for k, v in arrays.items()}
        print(f"  wrote {name} ({os.path.getsize(path) / 1e3:.0f} kB)")

    def check_restatements(self, tag, f1, f2, coords, L, r, legacy, ref_out, rows=None):
        """torch_cpu must be bit-identical; the C oracle within fp32 noise."""
        t1, t2, tc = (torch.from_numpy(a) for a in (f1, f2, coords))
        mine = torch_cpu.corr_lookup(t1, t2, tc, L, r, legacy).numpy()
        bitwise = bool(np.array_equal(mine, ref_out))
        if rows is None:
            orc_out = orc.corr_lookup(f1, f2, coords, L, r, legacy)
            err = orc.rel_err(orc_out, ref_out)
        else:
            orc_rows = orc.corr_lookup(f1, f2, coords, L, r, legacy, rows=rows)
            err = orc.rel_err(orc_rows, rows_of(ref_out, rows))
        rec = {"case": tag, "torch_cpu_bitwise": bitwise, "oracle_rel_err": err}
        self.meta["oracle_checks"].append(rec)
        print(f"    {tag}: torch_cpu bitwise={bitwise}  oracle rel err={err:.2e}")
        assert err < 2e-6, rec
        assert bitwise, rec

    # ------------------------------------------------------------------
    def sampler_kat(self):
        H, W, D = 8, 12, 16
        spike = (3, 7, 11)
        v = np.zeros((1, 1, H, W, D), np.float32)
        v[(0, 0) + spike] = 1.0
        q = [(3, 7, 11), (3, 11, 7), (3, 9, 11), (3, 7.25, 11), (3, 7, 10.5), (0, 0, 0), (7, 11, 15),
             (3.5, 7.5, 11.5), (-0.5, 7, 11), (8.2, 3, 3)]
        qa = np.array(q, np.float32).reshape(1, len(q), 1, 1, 3)
        imp = {}
        for leg in (False, True):
            imp[leg] = self.sampler(torch.from_numpy(v), torch.from_numpy(qa), legacy_wd_swap=leg).numpy()
        cube = np.zeros((1, 1, 16, 16, 16), np.float32)
        cube[0, 0, 3, 7, 11] = 1.0
        cq = np.array([(3, 7, 11), (3, 11, 7)], np.float32).reshape(1, 2, 1, 1, 3)
        cube_leg = self.sampler(torch.from_numpy(cube), torch.from_numpy(cq), legacy_wd_swap=True).numpy()
        # random volume, non-cubic, 2 channels, random points incl. out-of-range
        rv = prng.normal(101, (1, 2, 9, 7, 8))
        pts = np.stack([prng.uniform(102 + k, (1, 4, 5, 6), -1.5, s + 0.5) for k, s in enumerate((9, 7, 8))], -1)
        rnd = {leg: self.sampler(torch.from_numpy(rv), torch.from_numpy(pts), legacy_wd_swap=leg).numpy()
               for leg in (False, True)}
        for leg in (False, True):
            e = orc.rel_err(orc.sample(rv, pts, leg), rnd[leg])
            self.meta["oracle_checks"].append({"case": f"sampler_random_legacy{int(leg)}", "oracle_rel_err": e})
            assert e < 1e-6
            assert np.array_equal(orc.sample(v, qa, leg).astype(np.float32), imp[leg])
        self.save("sampler_kat.npz", imp_queries=qa, imp_fixed=imp[False], imp_legacy=imp[True],
                  cube_queries=cq, cube_legacy=cube_leg, rand_seed=np.array([101, 102, 103, 104]),
                  rand_pts=pts, rand_fixed=rnd[False], rand_legacy=rnd[True])

    def peak_shift(self):
        G, C, shift = 16, 32, (1, 2, -1)
        f2 = prng.normal(201, (1, C, G, G, G))
        f1 = np.roll(f2, tuple(-s for s in shift), axis=(2, 3, 4)).copy()
        coords = prng.identity_coords(1, G, G, G)
        probes = np.array([(8, 8, 8), (8, 10, 5), (8, 12, 6), (7, 5, 11)], np.int64)
        res = {}
        for leg in (False, True):
            out = self.CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=1, radius=4,
                                 legacy_wd_swap=leg)(torch.from_numpy(coords)).numpy()
            res[leg] = np.stack([out[0, :, h, w, d] for (h, w, d) in probes])
            self.check_restatements(f"peak_legacy{int(leg)}", f1, f2, coords, 1, 4, leg, out)
        self.save("peak_shift.npz", seed=np.array([201]), G=np.array([G]), C=np.array([C]),
                  shift=np.array(shift), probes=probes, out_fixed=res[False], out_legacy=res[True])

    def corr_case(self, name, B, C, shape, L, r, max_flow, seed, nrows, store_pyr_rows=4, check=True):
        H, W, D = shape
        f1 = prng.normal(seed, (B, C, H, W, D))
        f2 = prng.normal(seed + 1, (B, C, H, W, D))
        coords = prng.flow_coords(seed + 2, B, H, W, D, max_flow)
        N = H * W * D
        rows = sample_rows(seed + 3, B * N, nrows)
        prow = rows[:store_pyr_rows]
        payload = dict(seeds=np.array([seed, seed + 1, seed + 2, seed + 3]),
                       shape=np.array([B, C, H, W, D, L, r]), max_flow=np.array([max_flow]), rows=rows)
        t0 = time.time()
        for leg in (False, True):
            blk = self.CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r,
                                 legacy_wd_swap=leg)
            out = blk(torch.from_numpy(coords)).numpy()
            tag = "legacy" if leg else "fixed"
            payload[f"out_rows_{tag}"] = rows_of(out, rows)
            payload[f"checksum_{tag}"] = checksums(out)
            payload[f"level_sums_{tag}"] = out.reshape(B, L, -1).astype(np.float64).sum(axis=(0, 2))
            if not leg:
                pyr = [p.numpy().reshape(B * N, -1) for p in blk.corr_pyramid]
                payload["pyr_rows"] = np.concatenate([p[prow] for p in pyr], axis=1).astype(np.float32)
                payload["pyr_checksum"] = np.stack([checksums(p) for p in pyr])
            if check:
                self.check_restatements(f"{name}_{tag}", f1, f2, coords, L, r, leg, out,
                                        rows=None if B * N <= 4096 else rows)
        print(f"    {name}: reference time {time.time() - t0:.1f}s")
        self.save(name + ".npz", **payload)

    def plumbing(self, ref_root):
        """Config #1: capture the fmaps/coords the RAFTDVC forward feeds CorrBlock."""
        from src.core.raft_dvc import RAFTDVC, RAFTDVCConfig  # type: ignore
        import src.core.raft_dvc as rd  # type: ignore
        torch.manual_seed(1234)
        cfg = RAFTDVCConfig(encoder_type="1/8", corr_levels=4, corr_radius=4, iters=12)
        model = RAFTDVC(cfg).eval()
        vol0 = torch.from_numpy(prng.uniform(301, (1, 1, 64, 64, 64)))
        vol1 = torch.roll(vol0, shifts=(2, -1, 3), dims=(2, 3, 4))
        captured = {"coords": [], "out": []}
        Orig = rd.CorrBlock

        class Spy(Orig):  # records inputs/outputs, behaviour unchanged
            def __init__(self, fmap1, fmap2, *a, **k):
                captured["fmap1"] = fmap1.detach().numpy().copy()
                captured["fmap2"] = fmap2.detach().numpy().copy()
                super().__init__(fmap1, fmap2, *a, **k)

            def __call__(self, coords):
                o = super().__call__(coords)
                captured["coords"].append(coords.detach().numpy().copy())
                captured["out"].append(o.detach().numpy().copy())
                return o

        rd.CorrBlock = Spy
        try:
            with torch.no_grad():
                flow_lo, flow_up = model(vol0, vol1, test_mode=True)
        finally:
            rd.CorrBlock = Orig
        coords = np.stack(captured["coords"])        # (12, 1, 3, 8, 8, 8)
        outs = np.stack(captured["out"])             # (12, 1, 2916, 8, 8, 8)
        rows = sample_rows(305, 512, 16)
        out_rows = np.stack([rows_of(o, rows) for o in outs])
        self.check_restatements("plumbing_iter0", captured["fmap1"], captured["fmap2"], coords[0], 4, 4, False, outs[0])
        self.save("plumbing.npz", fmap1=captured["fmap1"], fmap2=captured["fmap2"], coords=coords, rows=rows,
                  out_rows=out_rows, out_checksums=np.stack([checksums(o) for o in outs]),
                  flow_lo=flow_lo.numpy(), flow_up_checksum=checksums(flow_up.numpy()))

    def run(self, ref_root):
        print("sampler KATs");  self.sampler_kat()
        print("peak shift");    self.peak_shift()
        print("equivalence grid (B=2, C=16, 8^3)")
        for L in (1, 2, 4):
            for r in (3, 4):
                self.corr_case(f"equiv_L{L}_r{r}", 2, 16, (8, 8, 8), L, r, 1.0, 1000 + 10 * L + r, 16, 2)
        print("edge cases")
        self.corr_case("edge_978_L3_r3", 2, 8, (9, 7, 8), 3, 3, 4.0, 2000, 24)
        self.corr_case("edge_965_L2_r4", 1, 8, (9, 6, 5), 2, 4, 3.0, 2010, 24)
        self.corr_case("edge_882_L2_r2", 1, 8, (8, 8, 2), 2, 2, 2.0, 2020, 24)   # level 1 is (4,4,1): zero level
        self.corr_case("edge_888_L4_r4", 1, 8, (8, 8, 8), 4, 4, 2.0, 2030, 24)   # level 3 is 1^3: zero level
        print("BASELINE configs")
        self.corr_case("cfg2", 1, 128, (16, 16, 16), 4, 4, 2.0, 3000, 128)
        self.corr_case("cfg3", 1, 128, (32, 32, 32), 4, 4, 2.0, 3100, 96, store_pyr_rows=2)
        print("plumbing (RAFTDVC 64^3, 1/8, L=4, 12 iters)")
        self.plumbing(ref_root)
        with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
            json.dump(self.meta, f, indent=1, default=float)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    Gen(a.reference).run(a.reference)
