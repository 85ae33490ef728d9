#!/bin/bash
# A/B of the current libdvccorr.so against ab/libdvccorr_base.so (bench + lookup PMC); parity subset first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2j}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_proj.py -q --timeout 300 --timeout-method thread -x > "$OUT/t.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/t.log"; grep -E "^FAILED" "$OUT/t.log" | head -5
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
for i in 1 2; do
  b new$i python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} || exit 3
  DVCCORR_LIB=$R/ab/libdvccorr_base.so b base$i python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} || exit 3
done
b new_fp32 python -u bench.py --no-cpu-baseline --precision fp32 || exit 3
cd "$R"
TAG=${TAG:-r2j} VARIANT=2 PMC_GROUPS="FETCH_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" EXTRA="--reps 2" bash tools/pmc_groups.sh || exit 3
exit 0
