#!/bin/bash
# Round 6: does the lookup reuse lines across consecutive lookups (L2 / Infinity Cache)?  Bench lines with every
# lookup at the same coordinates (--coord-fields 1) against the metric's 12 fields, the plane loads' cache policies
# (tuning lookup_ldpol), and the counters this rocprofv3 offers for memory-side (MALL / DRAM) traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6k; mkdir -p $OUT
export TMPDIR=/tmp
one() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])"
}
for i in 1 2; do
  one f12_$i
  one f1_$i --coord-fields 1
  one f2_$i --coord-fields 2
done
for p in 1 2 3; do one ldpol$p --tune lookup_ldpol=$p; done
timeout -k 10 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1; echo "list rc=$?"
grep -i -E "mall|dram|TCC_EA0_RDREQ|EA_RDREQ|TCC_BUBBLE|TCC_EA0_WRREQ" $OUT/list_avail.txt | head -40
