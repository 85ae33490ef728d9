#!/bin/bash
# Round 6: unconditional plane loads + the convc1 lookup's cross-level prefetch (XLP) -- GPU tests of the tile
# kernels, then alternating A/B bench lines: product (XLP on), libdvccorr_x0.so (XLP off), libdvccorr_base.so (HEAD
# before the change), for --convc1 and the default line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_proj.py tests/test_gpu_proj_grad.py tests/test_gpu_epe.py tests/test_gpu_parity.py tests/test_gpu_bricked.py tests/test_gpu_scale.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; grep -E "^FAILED" $OUT/pytest.log | head -5; [ $rc -ne 0 ] && exit $rc
L=raft-dvc_amd/dvccorr
one() {  # name lib args...
  local name=$1 lib=$2; shift 2
  DVCCORR_LIB=$PWD/$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])"
}
for i in 1 2; do
  one c_xlp_$i libdvccorr.so --convc1
  one c_x0_$i libdvccorr_x0.so --convc1
  one c_base_$i libdvccorr_base.so --convc1
done
for i in 1 2; do
  one n_new_$i libdvccorr.so
  one n_base_$i libdvccorr_base.so
done
timeout -k 10 200 python -u tools/trace_proj.py > $OUT/trace_proj.json 2> $OUT/trace_proj.err || { tail -3 $OUT/trace_proj.err; exit 3; }
python3 -c "
import json; d=json.load(open('$OUT/trace_proj.json')); print('trace event', d['event_ms'], 'end', d['end_us'])
for k in ('level_pos0','level_pos1','level_pos2','level_pos3'): print(k, {kk: v[1] for kk, v in d[k].items()})"
