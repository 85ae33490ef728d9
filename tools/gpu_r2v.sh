#!/bin/bash
# Round 2: f32 build with the next target tile prefetched -- fp32 parity tests, config #2 and the fp32 #3 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/${TAG:-r2v}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_backward.py tests/test_gpu_epe.py tests/test_gpu_proj.py -m gpu -q --timeout 300 --timeout-method thread -x > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
b() { local name=$1; shift; timeout -k 10 400 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?;
      echo "$name rc=$rc"; python -c "import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print(round(d['ms_per_step'],4), round(d['value']/1e6,1), 'M/s lookup', d['lookup_avg_ms'], 'build', d['build'], r['kernel'], r['frac'])" 2>/dev/null; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi; return $rc; }
b c2 python -u bench.py --size 16 --encoder 8 --precision fp32 --no-cpu-baseline || exit 3
b n1_fp32 python -u bench.py --precision fp32 --no-cpu-baseline || exit 3
exit 0
