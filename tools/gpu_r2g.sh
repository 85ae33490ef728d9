#!/bin/bash
# Round-2 GPU session G: tile lookup variants (branchless staging, columns per wave) A/B + parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2g}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "tile or cfg3 or variants or small_cases" > "$OUT/t.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/t.log"
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
for c in 3 2 1; do
  b n1_c$c python -u bench.py --no-cpu-baseline --tune lookup_cols=$c || exit 3
  b s8_c$c python -u bench.py --no-cpu-baseline --shard-of 8 --tune lookup_cols=$c || exit 3
done
b n1_c3_again python -u bench.py --no-cpu-baseline || exit 3
exit 0
