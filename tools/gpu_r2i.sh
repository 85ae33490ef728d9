#!/bin/bash
# Round-2 GPU session I: conflict-free LDS column reads in k_lookup_tile: parity + A/B vs ab/libdvccorr_base.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2i}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_proj.py tests/test_gpu_scale.py -q --timeout 300 --timeout-method thread -x > "$OUT/t.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/t.log"; grep -E "^FAILED|Error" "$OUT/t.log" | head -5
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; cat "$OUT/$name.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
for i in 1 2; do
  b new$i python -u bench.py --no-cpu-baseline || exit 3
  DVCCORR_LIB=$R/ab/libdvccorr_base.so b base$i python -u bench.py --no-cpu-baseline || exit 3
done
b new_s8 python -u bench.py --no-cpu-baseline --shard-of 8 || exit 3
b new_fp32 python -u bench.py --no-cpu-baseline --precision fp32 || exit 3
DVCCORR_LIB=$R/ab/libdvccorr_base.so b base_fp32 python -u bench.py --no-cpu-baseline --precision fp32 || exit 3
cd "$R"
TAG=r2i VARIANT=2 PMC_GROUPS="FETCH_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" EXTRA="--reps 2" bash tools/pmc_groups.sh || exit 3
exit 0
