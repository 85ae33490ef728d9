# PMC of the backward kernels at config #3 (bf16)
cd /tmp
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r3u; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum" "TA_BUSY_avr TA_TA_BUSY_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python $R/tools/bwd_only.py > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
