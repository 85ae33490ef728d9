#!/bin/bash
# One GPU-box session, steps chosen by STEPS (space list, run in order, stop at the first failure):
#   tests   -m gpu suite (one process) + smoke
#   bench   bench.py default line (config #3, the BASELINE metric) + the secondary lines in BENCH_SET
#   prof    rocprofv3 --kernel-trace --stats of the default bench line (PROF_ARGS), then of each "name|args" entry
#           of PROF_SET
#   pmc     rocprofv3 --pmc passes of the default lookup (tools/pmc_groups.sh; PMC_GROUPS overrides)
#   bwd     rocprofv3 kernel stats of the backward (tools/prof_bwd.sh), then its PMC passes (tools/pmc_bwd.sh,
#           groups in BWD_PMC_GROUPS; skipped when empty)
#   diag    build nothing; checks that libdvccorr_diag.so (make -C raft-dvc_amd/csrc diag) is present for the
#           A/B tools that need diagnostics knobs
#   cmd     an arbitrary command in $CMD (A/B scripts), under its own timeout
# Never retries a GPU step; a fault / abort / timeout ends the session.
#   TAG=r3a STEPS="tests bench" bash tools/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
T=${TAG:-r3}
OUT=$R/gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|Memory access fault" "$1"; }

b() {   # one bench line: name, args...
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?
  echo "bench $name rc=$rc"
  python - "$OUT/$name.json" <<'EOF' 2>/dev/null
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print(" ", round(d["ms_per_step"], 4), "ms", round(d["value"] / 1e6, 1), "M/s | lookup", d["lookup_avg_ms"],
      "ms frac", r["frac"], r["bound"], "| build", d["build"], "| cpu", (d.get("cpu_baseline") or {}).get("value"))
EOF
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; fi
  return $rc
}

for s in ${STEPS:-tests bench}; do
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=${MAXFAIL:-1} -v --timeout 300 --timeout-method thread \
        ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head
    if [ $rc -ne 0 ] || fault "$OUT/pytest.log"; then echo "STOP after pytest"; exit 3; fi
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -4 "$OUT/smoke.log"
    if [ $rc -ne 0 ]; then echo "STOP after smoke"; exit 3; fi ;;
  bench)
    b n1 ${N1_ARGS:-} || exit 3
    IFS=';' read -ra SET <<< "${BENCH_SET:-}"
    for e in "${SET[@]}"; do
      [ -z "$e" ] && continue
      name=${e%%|*}; args=${e#*|}
      b "$name" $args || exit 3
    done ;;
  prof)
    ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_n1" -o run \
        -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 ${PROF_ARGS:-} > "$OUT/prof_n1.log" 2>&1 ) \
        || { echo "rocprof failed"; tail -3 "$OUT/prof_n1.log"; exit 3; }
    echo "rocprof ok"
    IFS=';' read -ra SET <<< "${PROF_SET:-}"   # more profiled lines: "name|bench args;..." -> prof_<name>/
    for e in "${SET[@]}"; do
      [ -z "$e" ] && continue
      name=${e%%|*}; args=${e#*|}
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
          -- python "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 $args > "$OUT/prof_$name.log" 2>&1 ) \
          || { echo "rocprof $name failed"; tail -3 "$OUT/prof_$name.log"; exit 3; }
      echo "rocprof $name ok"
    done ;;
  pmc)
    TAG=$T VARIANT=2 PMC_GROUPS="${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT}" \
        EXTRA="${PMC_EXTRA:---reps 2}" bash tools/pmc_groups.sh || exit 3 ;;
  bwd)
    TAG=${T}_bwd bash tools/prof_bwd.sh || exit 3
    if [ -n "${BWD_PMC_GROUPS:-}" ]; then TAG=${T}_bwdpmc PMC_GROUPS="$BWD_PMC_GROUPS" bash tools/pmc_bwd.sh || exit 3; fi ;;
  diag)
    [ -f raft-dvc_amd/dvccorr/libdvccorr_diag.so ] || { echo "libdvccorr_diag.so missing (make -C raft-dvc_amd/csrc diag)"; exit 3; } ;;
  cmd)
    timeout -k 10 ${CMD_TIMEOUT:-600} bash -c "$CMD" > "$OUT/cmd.log" 2>&1; rc=$?
    echo "cmd rc=$rc"; tail -${CMD_TAIL:-40} "$OUT/cmd.log"
    if [ $rc -ne 0 ]; then exit 3; fi ;;
  esac
done
exit 0
