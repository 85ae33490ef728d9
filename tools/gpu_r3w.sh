for L in abl1 abl2 abl4; do TAG=bwp_$L DVCCORR_LIB=$PWD/raft-dvc_amd/dvccorr/libdvccorr_$L.so bash tools/prof_bwd.sh || exit 3; done
