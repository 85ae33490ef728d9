set -u
for cfg in "--shape 8,12,10 --levels 2 --radius 3 --channels 160" "--shape 8,12,10 --levels 2 --radius 3 --channels 128" "--shape 8,12,10 --levels 2 --radius 4 --channels 128" "--shape 8,12,16 --levels 2 --radius 3 --channels 128" "--shape 8,8,8 --levels 1 --radius 3 --channels 128"; do
  echo "== $cfg"
  DVCCORR_LIB=raft-dvc_amd/dvccorr/libdvccorr_head.so timeout -k 5 60 python tools/ab_bwd.py $cfg --reps 2 --save /tmp/a.pt > /dev/null || exit 3
  timeout -k 5 60 python tools/ab_bwd.py $cfg --reps 2 --compare /tmp/a.pt || exit 3
done
