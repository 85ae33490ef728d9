# order 0 vs order 1 window keys of the #5 convc1 path: L2 / fabric counters
cd $GRAFT_REPO_ROOT
for o in 0 1; do
  TAG=r3m VARIANT=2 SIZE=128 PREC=bf16 TUNE=fused_order=$o EXTRA="--reps 2 --levels 2 --impl fused --convc1" \
    PMC_GROUPS="TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
    bash tools/pmc_groups.sh || exit 1
done
