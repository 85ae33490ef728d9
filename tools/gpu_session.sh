#!/bin/bash
# One GPU-box session: parity tests, benches (materialised 32^3 = the headline line,
# fused 32^3, fused 128^3 L=2 = config #5's per-GPU shape), rocprofv3 kernel stats.
# Stops at the first fault / abort / timeout; never retries a GPU step.
#   TAG=r1c bash tools/gpu_session.sh        (SKIP_TESTS=1 / SKIP_PROF=1 to skip parts)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r1c}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault" "$1"; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
  if bad $rc || fault "$OUT/pytest.log"; then echo "STOP after pytest"; exit 3; fi
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"
  if bad $rc || fault "$OUT/smoke.log"; then echo "STOP after smoke"; exit 3; fi
fi

run_bench() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?
  echo "bench $name rc=$rc"; cat "$OUT/bench_$name.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/bench_$name.err"; exit 3; fi
}
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  run_bench mat32 ${BENCH_ARGS:-}
  run_bench fused32 --impl fused --no-cpu-baseline
  run_bench fused128 --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1
fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  for cfg in "mat32|" "fused32|--impl fused" "fused128|--impl fused --size 128 --encoder 2 --levels 2 --steps 2 --warmup 1"; do
    name=${cfg%%|*}; args=${cfg#*|}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
        -- python "$R/bench.py" --no-cpu-baseline $args > "$OUT/prof_$name.log" 2>&1
    rc=$?; echo "rocprof $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 "$OUT/prof_$name.log"; exit 3; fi
  done
fi
exit 0
