#!/bin/bash
# Round-2 GPU session K: convc1 fused into the on-the-fly lookup (k_fused_proj): parity tests, then
# config #5 bench lines (fused lookup + convc1 fused / unfused) and kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2k}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_proj_fused.py tests/test_gpu_proj.py -v --timeout 200 --timeout-method thread -x > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" "$OUT/pytest.log" | tail -40
if [ $rc -ne 0 ]; then tail -40 "$OUT/pytest.log"; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b f128_proj python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --convc1 fused --no-extras || exit 3
b f128_unf python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --convc1 unfused --no-extras || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python "$R/bench.py" --impl fused --size 128 --encoder 2 --levels 2 --steps 2 --warmup 1 --no-cpu-baseline --convc1 fused --no-extras --no-graph > "$OUT/prof.log" 2>&1
echo "rocprof rc=$?"
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))
for r in rows[:10]:
    print('%-90s %6s %10.1f us avg' % (r['Name'][:90], r['Calls'], float(r['AverageNs'])/1e3))
"
exit 0
