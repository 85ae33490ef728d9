#!/bin/bash
# Repeat runs after the splat2 fix: the full GPU suite twice, then the two convc1-fused test files five times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2rep}
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/suite$i.log" 2>&1; rc=$?
  echo "suite $i rc=$rc: $(tail -1 $OUT/suite$i.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_proj_fused.py tests/test_gpu_proj.py -q --timeout 120 --timeout-method thread > "$OUT/proj$i.log" 2>&1; rc=$?
  echo "proj $i rc=$rc: $(tail -1 $OUT/proj$i.log)"; [ $rc -eq 0 ] || exit $rc
done
