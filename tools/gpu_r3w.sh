TAG=r3w STEPS="tests bench prof" bash tools/gpu_session.sh || exit 3
TAG=bwp8 bash tools/prof_bwd.sh || exit 3
LIBS="main split3" TESTS=0 TAG=bw9 bash tools/gpu_bwd_many.sh || exit 3
for L in abl1 abl2 abl4; do TAG=bwp_$L DVCCORR_LIB=raft-dvc_amd/dvccorr/libdvccorr_$L.so bash tools/prof_bwd.sh || exit 3; done
