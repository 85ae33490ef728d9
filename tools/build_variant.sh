#!/bin/bash
# Link an A/B copy of libdvccorr with one source rebuilt under extra defines (the other objects from the product
# in-tree build):  bash tools/build_variant.sh backward qd2 -DDVC_QDEPTH=2  -> raft-dvc_amd/dvccorr/libdvccorr_qd2.so
set -eu
SRC=$1; NAME=$2; shift 2
cd "$(dirname "$0")/../raft-dvc_amd/csrc"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-result"
mkdir -p obj_ab
/opt/rocm/bin/hipcc $F "$@" -c $SRC.hip -o obj_ab/${SRC}_$NAME.o
/opt/rocm/bin/hipcc $F --hip-link -shared -o ../dvccorr/libdvccorr_$NAME.so $(ls obj/*.o | grep -v "obj/$SRC.o" | grep -v "obj/diag_") obj_ab/${SRC}_$NAME.o
echo "built libdvccorr_$NAME.so"
