#!/bin/bash
# Backward parity tests + backward timing (bench's backward block) + kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-bwd}
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_scale.py -q --timeout 300 --timeout-method thread -k "backward or grad or checkpoint or amp" > "$OUT/t.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/t.log"; grep -E "^FAILED" "$OUT/t.log" | head -5
if bad $rc; then echo STOP; exit $rc; fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['backward'])"
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))
for r in rows[:8]:
    print('%-80s %6s %10.1f us avg' % (r['Name'][:80], r['Calls'], float(r['AverageNs'])/1e3))
"
exit 0
