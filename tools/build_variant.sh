#!/bin/bash
# Link an A/B copy of libdvccorr with one or more sources rebuilt under extra defines (the other objects from the
# product in-tree build):  bash tools/build_variant.sh backward qd2 -DDVC_QDEPTH=2  -> raft-dvc_amd/dvccorr/libdvccorr_qd2.so
#                          bash tools/build_variant.sh fused_box,fused_proj wm -DDVC_FBOX_WMASK=1
set -eu
SRCS=$1; NAME=$2; shift 2
cd "$(dirname "$0")/../raft-dvc_amd/csrc"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-result"
mkdir -p obj_ab
OBJS=$(ls obj/*.o | grep -v "obj/diag_")
VOBJS=""
for SRC in ${SRCS//,/ }; do
  EXTRA=""
  [ "$SRC" = fused_proj ] && EXTRA=-fno-slp-vectorize   # as the Makefile
  /opt/rocm/bin/hipcc $F $EXTRA "$@" -c $SRC.hip -o obj_ab/${SRC}_$NAME.o &
  OBJS=$(echo "$OBJS" | grep -v "^obj/$SRC.o$")
  VOBJS="$VOBJS obj_ab/${SRC}_$NAME.o"
done
wait
/opt/rocm/bin/hipcc $F --hip-link -shared -o ../dvccorr/libdvccorr_$NAME.so $OBJS $VOBJS
echo "built libdvccorr_$NAME.so"
