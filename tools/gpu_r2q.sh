#!/bin/bash
# Round 2: config #5 on smooth vs i.i.d. synthetic flows (k_fused_box, k_fused_proj).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/${TAG:-r2q}
mkdir -p "$OUT"
b() { local name=$1; shift; timeout -k 10 400 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print(d['ms_per_step'], d['lookup_avg_ms'], r['frac'], r.get('mfma',{}).get('frac'))" ; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b f128_smooth python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --flow smooth || exit 3
b f128c_smooth python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --flow smooth --convc1 fused || exit 3
b n1_smooth python -u bench.py --no-cpu-baseline --flow smooth || exit 3
exit 0
