#!/usr/bin/env python3
"""Summaries from rocprofv3's SQLite output (run_results.db, the default format of this image).

    python tools/rocpd_summary.py stats <trace_dir> [--csv out.csv]
        per-kernel calls / total / average duration (ns), the --stats table
    python tools/rocpd_summary.py traffic <fetch_pass_dir> <write_pass_dir> --key KEY [--out profiles/traffic.json]
        HBM bytes per launch from two --pmc passes (FETCH_SIZE, WRITE_SIZE), corrected as
        tools/traffic.py does (MI355X_MICROARCH.md HBM section: FETCH_SIZE KB doubled for
        16-byte-per-lane reads on gfx950, WRITE_SIZE KB exact).
"""
import argparse
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def _dbs(d):
    return sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))


def stats(d):
    rows = defaultdict(lambda: [0, 0.0])
    for db in _dbs(d):
        c = sqlite3.connect(db)
        for name, calls, total in c.execute("select name, total_calls, total_duration from top_kernels"):
            rows[name][0] += calls
            rows[name][1] += total
    tot = sum(v[1] for v in rows.values()) or 1.0
    out = [(n, c, t, t / c, 100.0 * t / tot) for n, (c, t) in rows.items()]
    return sorted(out, key=lambda r: -r[2])


def pmc(d, counter):
    """Mean per dispatch of one counter, per kernel (summed over the counter's instances)."""
    per = defaultdict(lambda: defaultdict(float))
    for db in _dbs(d):
        c = sqlite3.connect(db)
        q = "select kernel_name, dispatch_id, value from counters_collection where counter_name = ?"
        for name, disp, val in c.execute(q, (counter,)):
            per[name][disp] += float(val)
    return {n: sum(v.values()) / len(v) for n, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("stats")
    s.add_argument("dir")
    s.add_argument("--csv")
    t = sub.add_parser("traffic")
    t.add_argument("fetch_dir")
    t.add_argument("write_dir")
    t.add_argument("--key", required=True)
    t.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "profiles", "traffic.json"))
    a = ap.parse_args()
    if a.cmd == "stats":
        rows = stats(a.dir)
        w = csv.writer(open(a.csv, "w") if a.csv else sys.stdout)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.0f}", f"{r[3]:.1f}", f"{r[4]:.2f}"])
        return
    fetch, write = pmc(a.fetch_dir, "FETCH_SIZE"), pmc(a.write_dir, "WRITE_SIZE")
    entry = {"note": "HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), rocprofv3 --pmc, gfx950"}
    for name in sorted(set(fetch) | set(write)):
        short = name.split("(")[0].replace("void ", "")
        fb, wb = 2 * fetch.get(name, 0.0) * 1024, write.get(name, 0.0) * 1024
        entry.setdefault("kernels", {})[short] = {"read_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
        if "k_lookup" in short:
            entry["lookup_hbm_bytes_per_launch"] = fb + wb
        if "k_build" in short:
            entry["build_hbm_bytes_per_launch"] = fb + wb
    data = json.load(open(a.out)) if os.path.exists(a.out) else {}
    data[a.key] = entry
    json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in entry.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
