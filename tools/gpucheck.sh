#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Stops at the first fault / abort / timeout (exit >= 124 or signal), but
# continues after ordinary pytest failures (exit 1) so the bench still runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ] || [ "$1" -ge 128 ]; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
      --maxfail=30 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  if bad $rc; then echo "STOP after pytest rc=$rc"; exit $rc; fi
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
  if bad $rc; then echo "STOP after smoke rc=$rc"; exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
  if bad $rc; then echo "STOP after bench rc=$rc"; exit $rc; fi
fi
if [ "${SKIP_PMC:-0}" != "1" ]; then
  cd /tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/pmc_$c" -o run \
        -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/$OUT/pmc_$c.log" 2>&1
    rc=$?; echo "pmc $c rc=$rc"
    if [ $rc -ne 0 ]; then cd "$GRAFT_REPO_ROOT"; exit $rc; fi
  done
  cd "$GRAFT_REPO_ROOT"
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
      -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc"; cd "$GRAFT_REPO_ROOT"
  find "$OUT/prof" -name "*stats*" | head
  if bad $rc; then exit $rc; fi
fi
exit 0
