# PMC of config #5's on-the-fly kernels (128^3 x 128 fmaps, L = 2, r = 4, bf16): k_fused_box and the convc1-fused path
cd $GRAFT_REPO_ROOT
for cv in "" "--convc1"; do
  TAG=r3k VARIANT=2 SIZE=128 PREC=bf16 EXTRA="--reps 2 --levels 2 --impl fused $cv" \
    PMC_GROUPS="FETCH_SIZE;WRITE_SIZE TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES" \
    bash tools/pmc_groups.sh || exit 1
  mv gpurun_out/r3k/pmcg_v2_bf16_128 gpurun_out/r3k/pmc128${cv:+_convc1}
done
