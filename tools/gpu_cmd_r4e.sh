#!/bin/bash
# round-4 session: backward + on-the-fly parity tests, config #5 fused lines + profile, fp16 / fp32 config #3
# lines, slab / full lookup timelines
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
timeout -k 10 900 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py tests/test_gpu_proj_fused.py \
    tests/test_gpu_amp.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r4e/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4e/pytest.log; [ $rc -eq 0 ] || exit 3
TAG=r4e STEPS="bench prof" N1_ARGS="--impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline" PROF_ARGS="--impl fused --size 128 --encoder 2 --levels 2 --steps 2 --warmup 1" BENCH_SET="f128c|--impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --convc1;f128h|--impl fused --size 128 --encoder 2 --levels 2 --steps 3 --warmup 1 --no-cpu-baseline --precision fp16;n1h|--precision fp16 --no-cpu-baseline;n1f|--precision fp32 --no-cpu-baseline;s8|--shard-of 8 --no-cpu-baseline" bash tools/gpu_session.sh || exit 3
timeout -k 10 120 python -u tools/trace_lookup.py --shard-of 8 > gpurun_out/r4e/trace8.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/trace_lookup.py > gpurun_out/r4e/trace1.log 2>&1 || exit 3
