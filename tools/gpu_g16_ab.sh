set -u
O=gpurun_out/r5m; mkdir -p $O
for p in bf16 fp16; do
  timeout -k 10 120 python tools/ab_bwd.py --precision $p --tune bwd_g16=0 --save /tmp/base_$p.pt > $O/ab_$p.txt 2>&1 || { cat $O/ab_$p.txt; exit 1; }
  timeout -k 10 120 python tools/ab_bwd.py --precision $p --tune bwd_g16=1 --compare /tmp/base_$p.pt >> $O/ab_$p.txt 2>&1 || { cat $O/ab_$p.txt; exit 1; }
  timeout -k 10 120 python tools/ab_bwd.py --precision $p --tune bwd_g16=0 >> $O/ab_$p.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/ab_bwd.py --precision $p --tune bwd_g16=1 >> $O/ab_$p.txt 2>&1 || exit 1
  cat $O/ab_$p.txt
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_amp.py tests/test_gpu_proj_grad.py tests/test_gpu_epe.py > $O/t.log 2>&1; tail -3 $O/t.log
