#!/bin/bash
# Round-2 GPU session D: EPE (fp16 convc1), proj tests, smoke, kernel-trace stats of the n1 and shard8 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2d}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_epe.py tests/test_gpu_proj.py tests/test_gpu_scale.py -v -s --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "EPE\[|FAILED|passed|failed" "$OUT/t.log"
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -4 "$OUT/smoke.log"
if bad $rc; then echo STOP; exit $rc; fi
cd /tmp
for cfg in "n1|" "shard8|--shard-of 8" "shard8_nograph|--shard-of 8 --no-graph"; do
  name=${cfg%%|*}; args=${cfg#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
      -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 $args > "$OUT/prof_$name.log" 2>&1
  rc=$?; echo "rocprof $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/prof_$name.log"; exit 3; fi
done
exit 0
