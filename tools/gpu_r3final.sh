#!/bin/bash
# Validate the working-tree backward against the last committed build (libdvccorr_head.so), then the closing
# session (tools/gpu_r3close.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/dbg_bwd.sh > gpurun_out/dbg_final.log 2>&1
LIBS="head main" TAG=bwfinal bash tools/gpu_bwd_many.sh || exit 3
bash tools/gpu_r3close.sh
