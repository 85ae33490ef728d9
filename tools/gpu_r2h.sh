#!/bin/bash
# Round-2 GPU session H: GPU suite, bench (with backward), kernel stats, PMC passes (build, lookup, fused box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2h}
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
b shard8 python -u bench.py --shard-of 8 --no-cpu-baseline || exit 3
b fused128 python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/prof_n1.log" 2>&1
echo "rocprof n1 rc=$?"
G="FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
cd "$R"
TAG=r2h VARIANT=2 PMC_GROUPS="$G" EXTRA="--reps 2" bash tools/pmc_groups.sh || exit 3
TAG=r2h VARIANT=2 SIZE=128 PMC_GROUPS="$G" EXTRA="--reps 1 --impl fused --levels 2" bash tools/pmc_groups.sh || exit 3
exit 0
