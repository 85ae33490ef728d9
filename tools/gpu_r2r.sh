#!/bin/bash
# Round 2: XCD-aware k_pack_pyramid -- parity tests, bench lines and kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -x > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/prof_n1.log" 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_f128" -o run \
    -- python "$R/bench.py" --impl fused --size 128 --encoder 2 --levels 2 --steps 2 --warmup 1 --no-cpu-baseline --no-graph > "$OUT/prof_f128.log" 2>&1 || exit 3
grep -h pack_pyramid "$OUT"/prof_*/run_kernel_stats.csv | cut -c1-160
exit 0
