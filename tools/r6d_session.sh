#!/bin/bash
# Round 6: level-1 bricking A/B (tuning brick_min_dp 16 vs 32) on the default bench line, then FETCH_SIZE /
# WRITE_SIZE passes for the convc1-fused lookup and the config #5 on-the-fly lookups (bf16, fp32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6d; mkdir -p $OUT
export TMPDIR=/tmp
one() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json,sys;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])"
}
for i in 1 2 3; do
  one base_$i
  one dp16_$i --tune brick_min_dp=16
done
R=$PWD
cd /tmp
pmc() {  # name counter extra...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/$OUT/pmc_$name/p_$ctr" -o run -- \
    python "$R/tools/lookup_only.py" --variant 2 --reps 2 "$@" > "$R/$OUT/pmc_${name}_$ctr.log" 2>&1 || { echo "pmc $name $ctr failed"; tail -3 "$R/$OUT/pmc_${name}_$ctr.log"; exit 3; }
  echo "pmc $name $ctr ok"
}
pmc convc1 FETCH_SIZE --convc1
pmc convc1 WRITE_SIZE --convc1
pmc dp16 FETCH_SIZE --tune brick_min_dp=16
pmc dp16 WRITE_SIZE --tune brick_min_dp=16
pmc fused128 FETCH_SIZE --impl fused --size 128 --levels 2
pmc fused128 WRITE_SIZE --impl fused --size 128 --levels 2
pmc fused128_fp32 FETCH_SIZE --impl fused --size 128 --levels 2 --precision fp32
pmc fused128_fp32 WRITE_SIZE --impl fused --size 128 --levels 2 --precision fp32
