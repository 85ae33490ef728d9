#!/bin/bash
# rocprofv3 --pmc passes (one run per group; groups separated by ';') over tools/lookup_only.py.
# usage: TAG=r01 VARIANT=2 TUNE=lookup_nt=1 PMC_GROUPS="A B;C D" bash tools/pmc_groups.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-r01}/pmcg_v${VARIANT:-2}${TUNE:+_$TUNE}_${PREC:-bf16}_${SIZE:-32}${SUFFIX:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
IFS=';' read -ra GRPS <<< "${PMC_GROUPS}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python "$R/tools/lookup_only.py" --variant ${VARIANT:-2} --tune "${TUNE:-}" --precision ${PREC:-bf16} --size ${SIZE:-32} ${EXTRA:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit $rc; fi
done
exit 0
