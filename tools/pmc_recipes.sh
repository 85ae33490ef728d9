#!/bin/bash
# The rocprofv3 --pmc recipes behind the profiles (profiles/r03/, profiles/r04/), one per name:
#   bash tools/pmc_recipes.sh r3e     (run on the GPU box from the repo root)
# r3c: lookup SQ instruction / LDS counters; r3e: lookup read-request sizes (128-B lines) and L2; r3j: the small
# launches (config #2 fp32 16^3); r3k: config #5 on-the-fly kernels (k_fused_box, convc1 path); r3m: #5 window-key
# orders; the backward kernels: tools/pmc_bwd.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
case "${1:-}" in
r4a)   # round 4: the headline lookup's HBM traffic (bench roofline.traffic) and its read-request sizes / LDS
  cd $R && TAG=r4a VARIANT=2 EXTRA="--reps 2" PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_WRREQ_64B_sum;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" bash tools/pmc_groups.sh
  ;;
r4i)   # round 4: instruction-cache and issue counters of the lookup at the small launches (one rank's 8-way slab of
       # config #3, config #2 fp32) and at config #3 whole
  ICG="SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  cd $R && TAG=r4i VARIANT=2 SUFFIX=_s8 EXTRA="--reps 4 --shard-of 8" PMC_GROUPS="$ICG" bash tools/pmc_groups.sh || exit 1
  cd $R && TAG=r4i VARIANT=2 SIZE=16 PREC=fp32 EXTRA="--reps 4" PMC_GROUPS="$ICG" bash tools/pmc_groups.sh || exit 1
  cd $R && TAG=r4i VARIANT=2 EXTRA="--reps 2" PMC_GROUPS="$ICG" bash tools/pmc_groups.sh || exit 1
  ;;
r4p)   # round 4: the backward's gradient kernels at config #3 (tools/bwd_only.py): HBM / L2, issue, LDS, addresser
  cd $R && TAG=r4p PMC_GROUPS="FETCH_SIZE;WRITE_SIZE TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" bash tools/pmc_bwd.sh
  ;;
r3c)
  cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/r3c_avail.txt 2>&1
  cd $R && TAG=r3c VARIANT=2 EXTRA="--reps 2" PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_LDS;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" bash tools/pmc_groups.sh
  ;;
r3e)
  cd $R && TAG=r3e VARIANT=2 EXTRA="--reps 2" PMC_GROUPS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum;FETCH_SIZE;WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" bash tools/pmc_groups.sh
  ;;
r3j)
  cd $R && TAG=r3j VARIANT=2 SIZE=16 PREC=fp32 EXTRA="--reps 2" PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY;FETCH_SIZE;WRITE_SIZE" bash tools/pmc_groups.sh
  cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3j/kt16 -o run -- python $R/tools/lookup_only.py --variant 2 --size 16 --precision fp32 --reps 5 > /dev/null 2>&1
  echo kt rc=$?
  ;;
r3k)
  cd $R
  for cv in "" "--convc1"; do
    TAG=r3k VARIANT=2 SIZE=128 PREC=bf16 EXTRA="--reps 2 --levels 2 --impl fused $cv" \
      PMC_GROUPS="FETCH_SIZE;WRITE_SIZE TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES" \
      bash tools/pmc_groups.sh || exit 1
    mv gpurun_out/r3k/pmcg_v2_bf16_128 gpurun_out/r3k/pmc128${cv:+_convc1}
  done
  ;;
r3m)
  cd $R
  for o in 0 1; do
    TAG=r3m VARIANT=2 SIZE=128 PREC=bf16 TUNE=fused_order=$o EXTRA="--reps 2 --levels 2 --impl fused --convc1" \
      PMC_GROUPS="TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
      bash tools/pmc_groups.sh || exit 1
  done
  ;;
*) echo "usage: $0 r4a|r4i|r4p|r3c|r3e|r3j|r3k|r3m"; exit 2 ;;
esac
