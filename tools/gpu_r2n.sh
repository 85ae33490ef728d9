#!/bin/bash
# Round-2 checkpoint: full GPU suite, smoke, bench lines (n1 default, #5 fused, #5 fused + convc1), rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2n}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; grep -E "^FAILED" "$OUT/pytest.log" | head -10
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 400 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; tail -c 1500 "$OUT/$name.json"; echo; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py || exit 3
b fused128 python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
b fused128_convc1 python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --convc1 fused || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/prof_n1.log" 2>&1
echo "rocprof n1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_f128" -o run \
    -- python "$R/bench.py" --impl fused --size 128 --encoder 2 --levels 2 --steps 2 --warmup 1 --no-cpu-baseline --no-graph > "$OUT/prof_f128.log" 2>&1
echo "rocprof f128 rc=$?"
exit 0
