#!/bin/bash
# config #3 step A/B of the build's output-store policy (tuning build_stpol: 1 = nontemporal, the default; 0 = plain),
# alternating processes
set -u
for i in 1 2 3; do
  for t in build_stpol=1 build_stpol=0; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --tune $t > /tmp/b.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$t', round(d['ms_per_step'],4), d['build']['avg_ms'], d['lookup_avg_ms'])"
  done
done
