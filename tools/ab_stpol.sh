set -u
mkdir -p gpurun_out/r5g
export DVCCORR_LIB=$PWD/raft-dvc_amd/dvccorr/libdvccorr_diag.so
for i in 1 2; do
for t in "lookup_stpol=-1" "lookup_stpol=0" "lookup_stpol=16"; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --tune "$t" > gpurun_out/r5g/b_${t}_$i.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['ms_per_step'], d['lookup_avg_ms'])" gpurun_out/r5g/b_${t}_$i.json "$t"
done; done
