#!/usr/bin/env python3
"""rocprofv3 --pmc pass directories -> one JSON of per-kernel counter means plus derived metrics.

    python tools/pmc_json.py <dir containing p1, p2, ...> --out profiles/r02_x.json [--note "..."]

Derived (MI355X_MICROARCH.md conventions): hbm_read_bytes = 2 x FETCH_SIZE x 1024 (FETCH_SIZE reports half
the bytes of wide coalesced reads on gfx950), hbm_write_bytes = WRITE_SIZE x 1024, mfma_busy =
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), lds_bank_conflict_frac =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, l2_hit = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--out", required=True)
ap.add_argument("--note", default="")
ap.add_argument("--filter", default="dvc::")
a = ap.parse_args()
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if a.filter and a.filter not in name:
            continue
        vals[name.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"_note": a.note}
for k, d in vals.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    m["_dispatches"] = max(len(v) for v in d.values())
    if "FETCH_SIZE" in m:
        m["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
        m["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        m["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        m["l2_hit"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1)
    out[k] = m
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
json.dump(out, open(a.out, "w"), indent=1)
for k, m in out.items():
    if k.startswith("_"):
        continue
    print(k, {x: round(m[x], 4) for x in ("mfma_busy", "lds_bank_conflict_frac", "l2_hit") if x in m},
          {x: f"{m[x] / 1e6:.1f} MB" for x in ("hbm_read_bytes", "hbm_write_bytes") if x in m})
