#!/bin/bash
# A/B of k_pack_pyramid's channels per workgroup (tuning "pack_cg": 0 = by size, 8 = eight): bench lines at the 8-way
# slab and the full config #3, alternating, same box; the pack kernel's rocprof average per setting.
set -u
O=gpurun_out/packcg; mkdir -p $O
for i in 1 2; do
  for v in 0 8; do
    for cfg in "shard8|--shard-of 8" "n1|"; do
      name=${cfg%%|*}; args=${cfg#*|}
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --tune pack_cg=$v $args > $O/${name}_cg${v}_$i.json 2> $O/${name}_cg${v}_$i.err || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4), d['build']['avg_ms'])" $O/${name}_cg${v}_$i.json $name cg=$v
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in 0 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cg$v -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 --shard-of 8 --tune pack_cg=$v > $O/prof_cg$v.log 2>&1 || exit 1
  echo "== pack_cg=$v"; python tools/rocpd_summary.py stats $O/prof_cg$v | grep -E "pack_pyramid|pack_queries" | cut -c1-160
done
