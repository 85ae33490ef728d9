set -u
for t in "" "split_ach=0" "split_ach=2" "split_ach=3" "lookup_waves=0" ""; do
  timeout -k 10 120 python bench.py --size 16 --precision fp32 --no-cpu-baseline --steps 20 --warmup 5 ${t:+--tune $t} > /tmp/c.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('/tmp/c.json').read().strip().splitlines()[-1]); print('$t', round(d['ms_per_step'],4), d['lookup_avg_ms'])"
done
