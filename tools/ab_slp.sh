#!/bin/bash
# A/B of -fno-slp-vectorize on fused_proj.hip (#5 with convc1 fused); abl/libdvccorr_slp.so is a hand-built variant.
set -u
mkdir -p gpurun_out/r2ab
for i in 1 2; do
for v in default slp; do
  if [ $v = slp ]; then export DVCCORR_LIB=$PWD/abl/libdvccorr_slp.so; else unset DVCCORR_LIB; fi
  timeout -k 10 300 python -u bench.py --impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --convc1 fused > gpurun_out/r2ab/$v$i.json 2>gpurun_out/r2ab/$v$i.err || exit 3
  python -c "import json; d=json.load(open('gpurun_out/r2ab/$v$i.json')); print('$v', d['ms_per_step'], d['lookup_avg_ms'])"
done; done
