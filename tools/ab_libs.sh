#!/bin/bash
# A/B the default lookup of two builds of libdvccorr (same ABI): alternating processes, ab_lookup.py each.
#   bash tools/ab_libs.sh raft-dvc_amd/dvccorr/libdvccorr_base.so raft-dvc_amd/dvccorr/libdvccorr.so [ab_lookup args]
set -u
A=$1; B=$2; shift 2
for i in 1 2 3; do
  for L in "$A" "$B"; do
    DVCCORR_LIB=$L timeout -k 5 120 python ${SCRIPT:-tools/ab_lookup.py} "$@" || exit 1
  done
done
