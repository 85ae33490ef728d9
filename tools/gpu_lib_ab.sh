#!/bin/bash
# backward A/B over builds of libdvccorr (tools/ab_bwd.py with DVCCORR_LIB), bitwise against the first, then the
# per-kernel times of each (rocprofv3 kernel stats):
#   LIBS="libdvccorr.so libdvccorr_ab_q4.so" PREC=bf16 ROUNDS=2 bash tools/gpu_lib_ab.sh
set -u
P=${PREC:-bf16}; N=${ROUNDS:-2}
D=raft-dvc_amd/dvccorr
first=""
for i in $(seq 1 $N); do
  for lib in $LIBS; do
    if [ -z "$first" ]; then
      DVCCORR_LIB=$D/$lib timeout -k 10 120 python tools/ab_bwd.py --precision $P --save /tmp/bwd_ref.pt 2>&1 | grep -v amdgpu.ids || exit 1
      first=$lib
    else
      DVCCORR_LIB=$D/$lib timeout -k 10 120 python tools/ab_bwd.py --precision $P --compare /tmp/bwd_ref.pt 2>&1 | grep -v amdgpu.ids || exit 1
    fi
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in $LIBS; do
  d=gpurun_out/libab_${lib%.so}
  DVCCORR_LIB=$D/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run -- python tools/ab_bwd.py --precision $P > $d.log 2>&1 || exit 1
  echo "== $lib"
  python tools/rocpd_summary.py stats $d | python -c '
import sys, csv
for r in list(csv.reader(sys.stdin))[1:]:
    if "grad_q" in r[0] or "grad_t" in r[0] or "win_grad" in r[0]:
        print(f"  {float(r[3]):8.1f} us  {r[0][:70]}")'
done
