#!/bin/bash
# rocprofv3 --pmc passes (one run per ';'-separated group) over tools/bwd_only.py (config #3 backward).
#   TAG=bwpmc PMC_GROUPS="SQ_WAVES SQ_BUSY_CYCLES;FETCH_SIZE" bash tools/pmc_bwd.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-bwpmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
IFS=';' read -ra GRPS <<< "${PMC_GROUPS}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python "$R/tools/bwd_only.py" --reps 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/p$i.log"; exit 3; fi
done
exit 0
