#!/bin/bash
# Round-2 GPU session A: existing GPU suite, then the new config #4/#5 + boundary tests, smoke, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2a}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail=20 \
    --ignore=tests/test_gpu_scale.py > "$OUT/pytest_old.log" 2>&1
rc=$?; echo "pytest old rc=$rc"; tail -4 "$OUT/pytest_old.log"
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_new.log" 2>&1
rc=$?; echo "pytest new rc=$rc"; grep -E "PASSED|FAILED|ERROR" "$OUT/pytest_new.log" | head -20
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -4 "$OUT/smoke.log"
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
exit 0
