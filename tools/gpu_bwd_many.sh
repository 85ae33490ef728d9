#!/bin/bash
# Backward A/B over several builds: LIBS="lds1 qd2 main qd4" (libdvccorr_<name>.so; main = the in-tree
# library), each timed by tools/ab_bwd.py and compared with the first; then (TESTS=1) the backward GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bwmany}
mkdir -p "$OUT"
export TMPDIR=/tmp
lib() { if [ "$1" = main ]; then echo raft-dvc_amd/dvccorr/libdvccorr.so; else echo raft-dvc_amd/dvccorr/libdvccorr_$1.so; fi; }
set -- $LIBS
first=$1
DVCCORR_LIB=$(lib $first) timeout -k 5 120 python tools/ab_bwd.py ${ARGS:-} --save /tmp/first.pt || exit 3
for rep in 1 2; do
  for n in $LIBS; do
    DVCCORR_LIB=$(lib $n) timeout -k 5 120 python tools/ab_bwd.py ${ARGS:-} --compare /tmp/first.pt || exit 3
  done
done
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TEST_FILES:-tests/test_gpu_backward.py} \
      > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
  [ $rc -eq 0 ] || exit 3
fi
exit 0
