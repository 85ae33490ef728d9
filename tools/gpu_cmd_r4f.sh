#!/bin/bash
# round-4 session: lookup parity tests with the 8-byte-chunk / three-plane pipeline, A/B against the
# 16-byte-chunk build (libdvccorr_cb16.so), slab and config #3 lines, timelines
set -u
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bricked.py tests/test_gpu_amp.py \
    tests/test_gpu_scale.py tests/test_gpu_proj.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 3
B=raft-dvc_amd/dvccorr/libdvccorr_cb16.so; M=raft-dvc_amd/dvccorr/libdvccorr.so
bash tools/ab_libs.sh $B $M --calls 20 > $O/ab_bf16.log 2>&1 || exit 3
bash tools/ab_libs.sh $B $M --calls 20 --convc1 > $O/ab_proj.log 2>&1 || exit 3
for L in $B $M $B $M; do
  DVCCORR_LIB=$L timeout -k 10 300 python -u bench.py --shard-of 8 --no-cpu-baseline --steps 20 >> $O/s8.jsonl 2>> $O/s8.err || exit 3
done
for L in $B $M; do
  DVCCORR_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline >> $O/n1.jsonl 2>> $O/n1.err || exit 3
done
timeout -k 10 120 python -u tools/trace_lookup.py --shard-of 8 > $O/trace8.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/trace_lookup.py > $O/trace1.log 2>&1 || exit 3
