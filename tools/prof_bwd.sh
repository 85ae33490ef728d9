#!/bin/bash
# rocprofv3 kernel trace of tools/ab_bwd.py (config #3 backward) into gpurun_out/$TAG
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG:-bwp}" -o run \
    -- python "$R/tools/ab_bwd.py" --reps 5 ${ARGS:-} > "$R/gpurun_out/${TAG:-bwp}.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
