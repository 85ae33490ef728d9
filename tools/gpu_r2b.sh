#!/bin/bash
# Round-2 GPU session B: GPU suite, default bench, per-rank diagnostics (--shard-of), 2-rank rehearsal, cfg #4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2b}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 \
    > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if bad $rc; then echo STOP; exit $rc; fi
fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py || exit 3
for n in 2 4 8; do b shard$n python -u bench.py --shard-of $n --no-cpu-baseline || exit 3; done
b shard8_nograph python -u bench.py --shard-of 8 --no-cpu-baseline --no-graph || exit 3
DVCCORR_BENCH_ONE_DEVICE=1 b rehearse2 python -u bench.py --gpus 2 --dist-backend gloo --cfg4-steps 0 --steps 5 || exit 3
b cfg4_n1 python -u bench.py --size 64 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
b cfg4_shard8 python -u bench.py --size 64 --steps 3 --warmup 1 --shard-of 8 --no-cpu-baseline || exit 3
exit 0
