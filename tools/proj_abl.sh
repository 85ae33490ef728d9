#!/bin/bash
# convc1-fused lookup (config #3) under diagnostics builds of lookup_tile_proj.hip (DVC_PROJ_ABL: 1 no weight loads,
# 2 no MFMAs), alternating processes; the outputs of the ablated builds are wrong by construction
set -u
for i in 1 2; do
  for lib in libdvccorr.so libdvccorr_pabl1.so libdvccorr_pabl2.so; do
    DVCCORR_LIB=raft-dvc_amd/dvccorr/$lib timeout -k 10 120 python bench.py --convc1 --no-cpu-baseline --steps 10 --warmup 3 > /tmp/p.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('/tmp/p.json').read().strip().splitlines()[-1]); print('$lib', round(d['ms_per_step'],4), d['lookup_avg_ms'])"
  done
done
