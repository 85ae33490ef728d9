#!/bin/bash
# Round 6: config #5 box kernel A/B of library builds, alternating bench.py processes (each lookup_avg_ms).
#   OUTDIR=r6n bash tools/r6n_session.sh libdvccorr_wmask.so [more variant libs]
# The first run (gpurun_out/r6n) also took the fused_ablate breakdown of this tree (diagnostics library):
#   python tools/ab_fused.py --size 128 --levels 2 --rounds 2 --reps 3 --variants 2,2:a1,2:a2,2:a4,2:a8,2:a12,2:a13
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUTDIR:-r6n}; mkdir -p $OUT
export TMPDIR=/tmp
L=raft-dvc_amd/dvccorr
one() {  # name lib args...
  local name=$1 lib=$2; shift 2
  DVCCORR_LIB=$PWD/$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --impl fused --size 128 --encoder 2 --levels 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['lookup_avg_ms'], d['roofline']['frac'])"
}
for i in $([ -n "${CONVC1_ONLY:-}" ] || echo 1 2); do
  one b_base_$i libdvccorr.so --steps 3 --warmup 1
  for v in "$@"; do
    one b_${v#libdvccorr_}_$i $v --steps 3 --warmup 1
  done
done
if [ -n "${CONVC1_ONLY:-}" ]; then   # the convc1 on-the-fly path only
  for i in 1 2 3; do
    for v in libdvccorr.so "$@"; do
      one c_${v#libdvccorr_}_$i $v --convc1 --steps 3 --warmup 1
    done
  done
  exit 0
fi
if [ -n "${MODES:-}" ]; then   # convc1 / fp32 instances too
  for i in 1 2; do
    for v in libdvccorr.so "$@"; do
      one c_${v#libdvccorr_}_$i $v --convc1 --steps 3 --warmup 1
      one f_${v#libdvccorr_}_$i $v --precision fp32 --steps 2 --warmup 1
    done
  done
fi
