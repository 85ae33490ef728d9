#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel (name filter), mean counter value per dispatch.

HBM bytes follow MI355X_MICROARCH.md: FETCH_SIZE (KB) reads 1/2 of wide coalesced
streaming reads on gfx950 (doubled here, flagged as 'fetch_x2'); WRITE_SIZE (KB) exact for
16-B stores (our 4-B-per-lane coalesced stores are uncalibrated)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if filt and filt not in name:
            continue
        key = (name[:70], r.get("Dispatch_Id"))
        vals[name[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
