#!/bin/bash
# Round-2 GPU session C: EPE loop, full GPU suite (row/level split + build chunking), per-rank diagnostics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2c}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_epe.py -v -s --timeout 200 --timeout-method thread > "$OUT/epe.log" 2>&1
rc=$?; echo "epe rc=$rc"; grep -E "EPE\[|PASSED|FAILED" "$OUT/epe.log"
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 \
    --ignore=tests/test_gpu_epe.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py --no-cpu-baseline || exit 3
for n in 2 4 8; do b shard$n python -u bench.py --shard-of $n --no-cpu-baseline || exit 3; done
exit 0
