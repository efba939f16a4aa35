#!/bin/bash
# Build a variant of libetcd_quorum.so with extra compile flags, reusing the
# main build's objects that the flags do not touch (copied with their
# timestamps, so make only rebuilds what depends on the changed sources).
#   scripts/build_variant.sh NAME "-DQE_PSTEP_TPB=4" [prog|all]
# -> etcd_amd/lib/variants/libetcd_quorum_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; WHAT=${3:-prog}
OBJ=$R/etcd_amd/build_$NAME
rm -rf "$OBJ"; mkdir -p "$OBJ" "$R/etcd_amd/lib/variants"
if [ "$WHAT" = prog ]; then
  cp -p "$R"/etcd_amd/build/qe_inst_[0-9]*.o "$R"/etcd_amd/build/qe_api.o "$R"/etcd_amd/build/qe_pack.o \
        "$R"/etcd_amd/build/qe_host.o "$R"/etcd_amd/build/qe_comm.o "$OBJ"/
fi
make -s -j8 -C "$R/etcd_amd/csrc" OBJDIR="$OBJ" LIBOUT="$R/etcd_amd/lib/variants/libetcd_quorum_$NAME.so" EXTRA="-DQE_VARIANT_BUILD $FLAGS"
