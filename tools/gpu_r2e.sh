#!/bin/bash
# Round-2 GPU session E: GPU suite (single-pass pack, split fix), benches, rehearsal, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2e}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if bad $rc; then echo STOP; exit $rc; fi
fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py || exit 3
for n in 2 4 8; do b shard$n python -u bench.py --shard-of $n --no-cpu-baseline || exit 3; done
DVCCORR_BENCH_ONE_DEVICE=1 b rehearse2 python -u bench.py --gpus 2 --dist-backend gloo --cfg4-steps 0 --steps 5 || exit 3
cd /tmp
for cfg in "n1|" "shard8|--shard-of 8"; do
  name=${cfg%%|*}; args=${cfg#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
      -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 $args > "$OUT/prof_$name.log" 2>&1
  rc=$?; echo "rocprof $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/prof_$name.log"; exit 3; fi
done
exit 0
