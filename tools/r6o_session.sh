#!/bin/bash
# Round 6: masked window writes in the box kernels -- fused / parity / AMP / scale GPU tests, then the config #5 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-r6o}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused_f32.py tests/test_gpu_parity.py tests/test_gpu_scale.py \
  tests/test_gpu_amp.py tests/test_gpu_proj_fused.py -m gpu --maxfail=3 -v --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; grep -E "^FAILED|^ERROR" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 3
one() {  # name args...
  local name=$1; shift
  timeout -k 10 500 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', round(d['ms_per_step'],4), 'ms lookup', d.get('lookup_avg_ms'), 'frac', r['frac'])"
}
one fused128 --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1
one fused128_fp32 --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 --precision fp32 --steps 2 --warmup 1
