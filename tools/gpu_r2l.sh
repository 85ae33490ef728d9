#!/bin/bash
# k_fused_proj ablations + PMC passes at config #5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r2l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_fproj.py > "$OUT/ab.log" 2>&1; rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.log"
[ $rc -ne 0 ] && exit $rc
G="FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
TAG=${TAG:-r2l} VARIANT=2 SIZE=128 PMC_GROUPS="$G" EXTRA="--reps 1 --impl fused --levels 2 --convc1" bash tools/pmc_groups.sh || exit 3
exit 0
