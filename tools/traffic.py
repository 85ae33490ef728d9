#!/usr/bin/env python3
"""HBM traffic per launch of the bench's kernels from two rocprofv3 --pmc passes.

    python tools/traffic.py <fetch_pass_dir> <write_pass_dir> --key materialised_bf16_32_L4_r4_n1 \
        [--out profiles/traffic.json]

Counters are corrected as MI355X_MICROARCH.md (HBM section) prescribes: FETCH_SIZE
(KB) reports half of the bytes of wide coalesced 16-byte-per-lane reads on gfx950 (the
tile lookup's plane loads and the build's operand loads are that shape), so it is
doubled; WRITE_SIZE (KB) is exact for the output stores (checked: the lookup's
WRITE_SIZE equals its output bytes to 0.1 %).  Values are means over dispatches."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--key", required=True)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "traffic.json"))
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_dir, "FETCH_SIZE")
    write = per_kernel(a.write_dir, "WRITE_SIZE")
    entry = {"note": "HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), rocprofv3 --pmc, gfx950"}
    for name in sorted(set(fetch) | set(write)):
        short = name.split("(")[0].replace("void ", "")
        fb = 2 * fetch.get(name, 0.0) * 1024
        wb = write.get(name, 0.0) * 1024
        entry.setdefault("kernels", {})[short] = {"read_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
        if "k_lookup" in short:
            entry["lookup_hbm_bytes_per_launch"] = fb + wb
        if "k_build" in short:
            entry["build_hbm_bytes_per_launch"] = fb + wb
    data = json.load(open(a.out)) if os.path.exists(a.out) else {}
    data[a.key] = entry
    json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
