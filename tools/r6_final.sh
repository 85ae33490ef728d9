#!/bin/bash
# Round-6 closing run on one box: the -m gpu suite + smoke, the bench lines (default = BASELINE config #3, then the
# secondary configurations), rocprofv3 kernel stats of the default line, PMC passes of the default lookup (one
# counter group per run), and the copy-rate probe (mixed read/write HBM rate on the same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r6z}; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; grep -E "^FAILED|^ERROR" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 3
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 3; }
  tail -4 $OUT/smoke.log
fi
one() {  # name args...
  local name=$1; shift
  timeout -k 10 500 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,1), 'M/s lookup', d.get('lookup_avg_ms'), 'frac', r['frac'], 'bwd', (d.get('backward') or {}).get('avg_ms'))"
}
one n1
one convc1 --no-cpu-baseline --convc1
one fp32 --no-cpu-baseline --precision fp32
one cfg2 --no-cpu-baseline --size 16 --encoder 8 --precision fp32
one shard8 --no-cpu-baseline --shard-of 8
one fused128 --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1
one fused128_fp32 --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 --precision fp32 --steps 2 --warmup 1
one fused128_convc1 --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 --convc1 --steps 3 --warmup 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
    -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/prof_n1.log" 2>&1 ) || { echo "rocprof failed"; exit 3; }
echo "rocprof ok"
cd /tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc/p$i" -o run -- \
      python "$R/tools/lookup_only.py" --variant 2 --reps 2 > "$OUT/pmc_p$i.log" 2>&1 || { echo "pmc $i failed"; exit 3; }
  echo "pmc pass $i ok"
done
cd "$R"
timeout -k 10 120 tools/probe/mix2_probe > $OUT/probe_mix2.txt 2>&1 || { echo "probe failed"; exit 3; }
grep -i "copy\|rd 1\|wr 1" $OUT/probe_mix2.txt | head -8
