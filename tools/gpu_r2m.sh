#!/bin/bash
# fused box port: parity tests (fused paths), then #5 timing of the box (variant 2) with ablations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2m}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_proj_fused.py tests/test_gpu_scale.py -q -x --timeout 300 --timeout-method thread -k "fused or cfg5" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" "$OUT/pytest.log" | head; exit $rc; }
timeout -k 10 300 python -u tools/ab_fused.py --size 128 --levels 2 --variants 2,2:a1,2:a2,2:a4,2:a8,2:a12,2:a13 --rounds 1 --reps 3 > "$OUT/ab_box.log" 2>&1; echo "ab_box rc=$?"; tail -2 "$OUT/ab_box.log"
timeout -k 10 300 python -u tools/ab_fproj.py --ablate 0 > "$OUT/ab_proj.log" 2>&1; tail -1 "$OUT/ab_proj.log"
exit 0
