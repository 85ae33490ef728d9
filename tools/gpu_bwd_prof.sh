#!/bin/bash
# per-kernel backward times (rocprofv3 --kernel-trace --stats over tools/ab_bwd.py, config #3) per dvc_set_tuning set:
#   SETS="bwd_gt_z2=0 bwd_gt_z2=1" PREC=bf16 TAG=z2 bash tools/gpu_bwd_prof.sh
set -u
P=${PREC:-bf16}; TAG=${TAG:-bp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for t in $SETS; do
  d=gpurun_out/${TAG}_$i
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run -- python tools/ab_bwd.py --precision $P --tune "$t" > $d.log 2>&1 || exit 1
  echo "== $t"; grep "backward median" $d.log
  python tools/rocpd_summary.py stats $d | python -c '
import sys, csv
rows = list(csv.reader(sys.stdin))[1:]
tot = 0.0
for r in rows:
    n, calls, avg = r[0], int(r[1]), float(r[3])
    if "dvc::" in n or "rocprim" in n:
        tot += avg * calls / 24
        print(f"  {avg:8.1f} us x{calls // 24:<3d} {n[:90]}")
print(f"  sum per backward {tot:.1f} us")'
  i=$((i+1))
done
