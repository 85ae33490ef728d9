#!/usr/bin/env python3
"""Print the kernels of the last dvc_corr_backward call in a rocprofv3 kernel trace (tools/prof_bwd.sh)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tr = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows), key=lambda x: x[1])
first = [i for i, t in enumerate(tr) if "k_win_grad" in t[0]][-1]
last = [i for i, t in enumerate(tr) if "k_unpack_sum" in t[0]][-1]
t0 = tr[first][1]
tot = {}
for n, a, b in tr[first:last + 1]:
    m = re.search(r"dvc::(\w+)", n)
    nm = m.group(1) if m else ("rocprim" if "rocprim" in n else n[:40])
    print(f"{nm:28s} start={(a - t0) / 1000:8.1f} dur={(b - a) / 1000:7.1f} us")
    tot[nm] = tot.get(nm, 0) + (b - a) / 1000
print("span", (tr[last][2] - t0) / 1000, "us;", {k: round(v, 1) for k, v in tot.items()})
