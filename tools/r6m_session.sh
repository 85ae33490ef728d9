#!/bin/bash
# Round 6: on-the-fly kernels with the 8 x 4 x 1 box group -- their GPU tests, then the config #5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_fused_f32.py tests/test_gpu_scale.py tests/test_gpu_amp.py tests/test_gpu_proj_fused.py \
    tests/test_gpu_backward.py -k "fused or cfg5 or fp32 or amp or grad_golden or Fused" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; grep -E "^FAILED" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 --steps 3 \
    --warmup 1 > $OUT/fused128.json 2> $OUT/fused128.err || { tail -5 $OUT/fused128.err; exit 3; }
python3 -c "import json;d=json.loads(open('$OUT/fused128.json').read().strip().splitlines()[-1]);print('fused128', d['ms_per_step'], d['lookup_avg_ms'], d['roofline']['frac'])"
