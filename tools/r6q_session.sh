#!/bin/bash
# Round 6, last tree: PMC passes of the config #5 on-the-fly lookups (bf16 k_fused_box, fp32 k_fused_box_f32) after
# the box group and the masked window writes, one counter group per run (traffic.json's #5 entries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6q; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
cd /tmp
pmc() {  # name counters extra...
  local name=$1 ctr=$2; shift 2
  local tag=${ctr%% *}
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/$OUT/pmc_$name/p_$tag" -o run -- \
    python "$R/tools/lookup_only.py" --variant 2 --reps 2 "$@" > "$R/$OUT/pmc_${name}_$tag.log" 2>&1 || { echo "pmc $name $tag failed"; tail -3 "$R/$OUT/pmc_${name}_$tag.log"; exit 3; }
  echo "pmc $name $tag ok"
}
pmc fused128 FETCH_SIZE --impl fused --size 128 --levels 2
pmc fused128 WRITE_SIZE --impl fused --size 128 --levels 2
pmc fused128 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES" --impl fused --size 128 --levels 2
pmc fused128 "SQ_VALU_MFMA_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" --impl fused --size 128 --levels 2
pmc fused128_fp32 FETCH_SIZE --impl fused --size 128 --levels 2 --precision fp32
pmc fused128_fp32 WRITE_SIZE --impl fused --size 128 --levels 2 --precision fp32
