#!/bin/bash
# Separate rocprofv3 --pmc passes (one counter group per run) over tools/lookup_only.py.
# usage: TAG=r01 VARIANT=0 bash tools/pmc.sh
#        PMC_GROUPS="FETCH_SIZE;SQ_WAVES SQ_BUSY_CYCLES" EXTRA="--impl fused --levels 2" SIZE=128 bash tools/pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r01}/pmc_v${VARIANT:-0}${TUNE:+_$TUNE}_${PREC:-bf16}_${SIZE:-32}${NAME:+_$NAME}
mkdir -p "$OUT"
export TMPDIR=/tmp
DEFAULT_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT;TCC_HIT_sum TCC_MISS_sum"
cd /tmp
i=0
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python "$R/tools/lookup_only.py" --variant ${VARIANT:-0} --tune "${TUNE:-}" --precision ${PREC:-bf16} --size ${SIZE:-32} ${EXTRA:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit $rc; fi
done
exit 0
