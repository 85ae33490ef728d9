#!/bin/bash
# Round 6: k_grad_t_dense on 4 x 4 x 8 target blocks (tuning bwd_bz8) -- backward GPU tests, then alternating timings of
# the config #3 backward (tools/ab_bwd.py) with the knob off / on, results compared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-r6bz8}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "^FAILED|^ERROR" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 3
fi
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/ab_bwd.py --save $OUT/off.pt > $OUT/off_$i.txt 2>&1 || { tail -3 $OUT/off_$i.txt; exit 3; }
  timeout -k 10 120 python -u tools/ab_bwd.py --tune bwd_bz8=1 --save $OUT/on.pt --compare $OUT/off.pt > $OUT/on_$i.txt 2>&1 || { tail -3 $OUT/on_$i.txt; exit 3; }
  grep median $OUT/off_$i.txt; grep median $OUT/on_$i.txt
done
rm -f $OUT/*.pt
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python $GRAFT_REPO_ROOT/tools/ab_bwd.py --tune bwd_bz8=1 --reps 5 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 3
