cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused_f32.py tests/test_gpu_scale.py::test_cfg5_fused_rows "tests/test_gpu_parity.py::test_small_cases_fp32" > gpurun_out/r6c/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6c/pytest.log; grep -E "^FAILED|Error" gpurun_out/r6c/pytest.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --impl fused --precision fp32 --size 128 --encoder 2 --levels 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r6c/f128_fp32.json 2> gpurun_out/r6c/f128_fp32.err || { tail -5 gpurun_out/r6c/f128_fp32.err; exit 3; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6c/f128_fp32.json').read().strip().splitlines()[-1]);print('fp32 mfma', d['ms_per_step'], d['lookup_avg_ms'], d['roofline'])"
timeout -k 10 500 python -u bench.py --impl fused --precision fp32 --size 128 --encoder 2 --levels 2 --steps 1 --warmup 1 --no-cpu-baseline --tune fused_variant=0 > gpurun_out/r6c/f128_fp32_valu.json 2> gpurun_out/r6c/f128_fp32_valu.err || { tail -5 gpurun_out/r6c/f128_fp32_valu.err; exit 3; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6c/f128_fp32_valu.json').read().strip().splitlines()[-1]);print('fp32 valu', d['ms_per_step'], d['lookup_avg_ms'], d['roofline'])"
