# PMC of the small launches: config #2 (16^3 fp32) and one rank's slab of an 8-way split at config #3 (bf16)
cd $GRAFT_REPO_ROOT && TAG=r3j VARIANT=2 SIZE=16 PREC=fp32 EXTRA="--reps 2" PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY;FETCH_SIZE;WRITE_SIZE" bash tools/pmc_groups.sh
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3j/kt16 -o run -- python $GRAFT_REPO_ROOT/tools/lookup_only.py --variant 2 --size 16 --precision fp32 --reps 5 > /dev/null 2>&1
echo kt rc=$?
