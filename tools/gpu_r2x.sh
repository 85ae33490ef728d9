#!/bin/bash
# Round-2 session x: the packed-FP32 op_sel fix of k_fused_proj (poison repro first), then the full GPU suite,
# PMC passes of the default (bricked) lookup and of its convc1-fused form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
T=${TAG:-r2x2}
OUT=$R/gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u tools/dbg_poison3.py 0 100 > "$OUT/poison3.log" 2>&1; rc=$?; echo "poison3 rc=$rc"; tail -3 "$OUT/poison3.log"
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head -10
if bad $rc; then echo STOP; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -4 "$OUT/smoke.log"
if bad $rc; then echo STOP; exit $rc; fi
b() { local name=$1; shift; timeout -k 10 400 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; python -c "import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print(round(d['ms_per_step'],4), round(d['value']/1e6,1), 'M/s lookup', d['lookup_avg_ms'], r['frac'], r.get('lookup'), (d.get('cpu_baseline') or {}).get('value'))" 2>/dev/null; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b n1 python -u bench.py || exit 3
b shard8 python -u bench.py --shard-of 8 --no-cpu-baseline || exit 3
b shard4 python -u bench.py --shard-of 4 --no-cpu-baseline || exit 3
b shard2 python -u bench.py --shard-of 2 --no-cpu-baseline || exit 3
b cfg4_n1 python -u bench.py --size 64 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
b n1_convc1 python -u bench.py --no-cpu-baseline --convc1 fused || exit 3
b n1_fp32 python -u bench.py --no-cpu-baseline --precision fp32 || exit 3
b cfg2_fp32 python -u bench.py --size 16 --encoder 8 --precision fp32 --no-cpu-baseline || exit 3
b fused128 python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline || exit 3
b fused128_convc1 python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --convc1 fused || exit 3
DVCCORR_BENCH_ONE_DEVICE=1 b rehearse2 python -u bench.py --gpus 2 --dist-backend gloo --cfg4-steps 0 --steps 5 || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/prof_n1.log" 2>&1 || exit 3
echo "rocprof n1 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg4" -o run \
    -- python "$R/bench.py" --size 64 --steps 2 --warmup 1 --no-cpu-baseline --no-graph > "$OUT/prof_cfg4.log" 2>&1 || exit 3
echo "rocprof cfg4 ok"
cd "$R"
G="FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
TAG=$T VARIANT=2 PMC_GROUPS="$G" EXTRA="--reps 2" bash tools/pmc_groups.sh || exit 3
TAG=$T VARIANT=2 TUNE=lookup_nt=1 PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" EXTRA="--reps 2 --convc1" bash tools/pmc_groups.sh || exit 3
TAG=$T VARIANT=2 PREC=fp32 PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" EXTRA="--reps 1" bash tools/pmc_groups.sh || exit 3
exit 0
