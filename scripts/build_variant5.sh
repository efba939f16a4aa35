#!/bin/bash
# Timing variant of libetcd_quorum.so where only the S = 5 Progress objects
# are rebuilt with extra flags (the bench's Progress workloads run S = 5):
#   scripts/build_variant5.sh NAME "-DQE_PSTEP_WAVES=4"
# OBJS="qe_inst_5 qe_inst_6" rebuilds those objects instead.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
OBJ=$R/etcd_amd/build_$NAME
rm -rf "$OBJ"; mkdir -p "$OBJ" "$R/etcd_amd/lib/variants"
cp -p "$R"/etcd_amd/build/*.o "$R"/etcd_amd/build/*.d "$OBJ"/
# the copied objects count as current (only the named ones are rebuilt, even
# when a header they include has changed since the main build)
touch "$OBJ"/*.o
for o in ${OBJS:-qe_inst_prog_5}; do rm -f "$OBJ/$o.o"; done
make -s -j8 -C "$R/etcd_amd/csrc" OBJDIR="$OBJ" LIBOUT="$R/etcd_amd/lib/variants/libetcd_quorum_$NAME.so" EXTRA="-DQE_VARIANT_BUILD $FLAGS"
