#!/bin/bash
# backward A/B over dvc_set_tuning knob sets (tools/ab_bwd.py, config #3), bitwise against the first set:
#   SETS="bwd_gt_cube=0 bwd_gt_cube=1" PREC=bf16 ROUNDS=2 bash tools/gpu_bwd_knobs.sh
set -u
P=${PREC:-bf16}; N=${ROUNDS:-2}
first=""
for i in $(seq 1 $N); do
  for t in $SETS; do
    if [ -z "$first" ]; then
      timeout -k 10 120 python tools/ab_bwd.py --precision $P --tune "$t" --save /tmp/bwd_ref.pt 2>&1 | grep -v amdgpu.ids || exit 1
      first=$t
    else
      timeout -k 10 120 python tools/ab_bwd.py --precision $P --tune "$t" --compare /tmp/bwd_ref.pt 2>&1 | grep -v amdgpu.ids || exit 1
    fi
  done
done
