#!/bin/bash
# A/B of dvc_set_tuning knob sets through bench.py (config #3 by default), alternating runs:
#   TAG=r5i ROUNDS=3 bash tools/ab_knob_bench.sh "lookup_lmix=0" "lookup_lmix=1" -- [extra bench args]
set -u
T=${TAG:-ab}; N=${ROUNDS:-3}
mkdir -p gpurun_out/$T
sets=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done; [ $# -gt 0 ] && shift
for i in $(seq 1 $N); do
  for t in "${sets[@]}"; do
    f=gpurun_out/$T/b_${t//[,=]/_}_$i.json
    timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 20 --tune "$t" "$@" > "$f" 2>/dev/null || exit 1
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])" "$f" "$t"
  done
done
