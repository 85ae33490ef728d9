#!/bin/bash
# Round 6: the convc1-fused lookup with the cross-level prefetch (XLP): its GPU tests, bench lines, timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_proj.py tests/test_gpu_proj_grad.py tests/test_gpu_epe.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; grep -E "^FAILED" $OUT/pytest.log | head -5; [ $rc -ne 0 ] && exit $rc
one() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])"
}
one convc1_1 --convc1
one convc1_2 --convc1
one convc1_fp32 --convc1 --precision fp32
one n1
timeout -k 10 200 python -u tools/trace_proj.py > $OUT/trace_proj.json 2> $OUT/trace_proj.err || { tail -3 $OUT/trace_proj.err; exit 3; }
python3 -c "
import json; d=json.load(open('$OUT/trace_proj.json')); print('trace event', d['event_ms'], 'end', d['end_us'])
for k in ('level_pos1','level_pos2','level_pos3'): print(k, d[k].get('prev_level_last_row->row0'), d[k].get('level_total(start->last_row)'))"
