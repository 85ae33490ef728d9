#!/bin/bash
# Round-2 GPU session F: pack_pyramid check + speed, lookup ablations (is the lookup read- or write-bound?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2f}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/t.log"
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py --no-cpu-baseline || exit 3
b shard8 python -u bench.py --shard-of 8 --no-cpu-baseline || exit 3
b abl_nostore python -u bench.py --no-cpu-baseline --tune lookup_ablate=1 || exit 3
b abl_noload python -u bench.py --no-cpu-baseline --tune lookup_ablate=2 || exit 3
b abl_none python -u bench.py --no-cpu-baseline --tune lookup_ablate=3 || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_shard8" -o run \
      -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 --shard-of 8 > "$OUT/prof_shard8.log" 2>&1
echo "rocprof rc=$?"
exit 0
