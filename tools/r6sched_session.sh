#!/bin/bash
# Round 6: hipcc scheduler strategies (-mllvm -amdgpu-sched-strategy=gcn-max-ilp / gcn-max-memory-clause) on the box
# kernel (config #5 bf16) and the bf16 tile lookup (config #3), alternating bench processes against the product library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6sched; mkdir -p $OUT
export TMPDIR=/tmp
L=raft-dvc_amd/dvccorr
one() {  # name lib args...
  local name=$1 lib=$2; shift 2
  DVCCORR_LIB=$PWD/$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'])"
}
for i in 1 2; do
  for v in libdvccorr.so libdvccorr_fbilp.so libdvccorr_fbmc.so; do
    one f_${v%.so}_$i $v --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1
  done
done
for i in 1 2 3; do
  for v in libdvccorr.so libdvccorr_ltilp.so libdvccorr_ltmc.so; do
    one m_${v%.so}_$i $v --steps 20 --warmup 5
  done
done
