#!/bin/bash
# Backward A/B on the GPU box: BASE (a libdvccorr_*.so build of the same ABI) vs the in-tree library, timed and
# compared by tools/ab_bwd.py (results and speed), then the backward GPU tests on the in-tree library.
#   BASE=raft-dvc_amd/dvccorr/libdvccorr_occ1.so TAG=bw2 bash tools/gpu_bwd_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bwab}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { timeout -k 5 120 python tools/ab_bwd.py "$@" || exit 3; }
DVCCORR_LIB=$BASE run --save /tmp/base.pt
run --compare /tmp/base.pt
DVCCORR_LIB=$BASE run
run
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TEST_FILES:-tests/test_gpu_backward.py} \
      > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
  [ $rc -eq 0 ] || exit 3
fi
exit 0
