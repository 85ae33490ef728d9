#!/bin/bash
# Round 6: the on-the-fly box kernels' XCD box group (8 x 4 x 1 against 4 x 4 x 2 boxes: ~11 % smaller level-0 union
# per XCD), alternating A/B at config #5; then the backward PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6l; mkdir -p $OUT
export TMPDIR=/tmp
L=raft-dvc_amd/dvccorr
one() {  # name lib args...
  local name=$1 lib=$2; shift 2
  DVCCORR_LIB=$PWD/$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])"
}
for i in 1 2; do
  one b_base_$i libdvccorr.so --steps 3 --warmup 1
  one b_g841_$i libdvccorr_g841.so --steps 3 --warmup 1
done
one f_base libdvccorr.so --precision fp32 --steps 2 --warmup 1
one f_g841 libdvccorr_g841f.so --precision fp32 --steps 2 --warmup 1
TAG=r6bwpmc PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS;SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" bash tools/pmc_bwd.sh
