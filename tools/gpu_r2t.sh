#!/bin/bash
# Round 2: DVC_BRICKED layout -- full GPU suite, brick A/B, bench lines bricked vs linear (DVCCORR_BRICKED=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2t}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head -20
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 300 python -u tools/ab_brick.py > "$OUT/ab_brick.log" 2>&1; rc=$?; echo "ab_brick rc=$rc"; tail -3 "$OUT/ab_brick.log"
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 400 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; python -c "import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print(round(d['ms_per_step'],4), round(d['value']/1e6,1), 'M/s lookup', d['lookup_avg_ms'], r['frac'], r.get('lookup'))" 2>/dev/null; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py --no-cpu-baseline || exit 3
DVCCORR_BRICKED=0 b n1_linear python -u bench.py --no-cpu-baseline || exit 3
b shard8 python -u bench.py --shard-of 8 --no-cpu-baseline || exit 3
DVCCORR_BRICKED=0 b shard8_linear python -u bench.py --shard-of 8 --no-cpu-baseline || exit 3
b cfg4 python -u bench.py --size 64 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
DVCCORR_BRICKED=0 b cfg4_linear python -u bench.py --size 64 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
b n1_convc1 python -u bench.py --no-cpu-baseline --convc1 fused || exit 3
DVCCORR_BRICKED=0 b n1_convc1_linear python -u bench.py --no-cpu-baseline --convc1 fused || exit 3
exit 0
