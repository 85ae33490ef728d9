#!/bin/bash
# Round-3 closing session on the GPU box: the -m gpu suite + smoke, the bench lines, the rocprof kernel stats of
# the default line, the backward kernel stats and its PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r3z STEPS="tests bench prof" BENCH_SET="fp32|--precision fp32;cfg2|--size 16 --precision fp32;shard8|--shard-of 8" \
    bash tools/gpu_session.sh || exit 3
TAG=bwpz bash tools/prof_bwd.sh || exit 3
TAG=bwpmcz PMC_GROUPS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr" \
    bash tools/pmc_bwd.sh || exit 3
exit 0
