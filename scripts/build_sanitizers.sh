#!/bin/bash
# Host-code sanitizer builds (the reference runs its tests
# with -race; the host C/C++ here gets ASan+UBSan and TSan):
#   etcd_amd/build_san/libetcd_quorum_asan.so  the library with qe_pack.cpp
#                                              under -fsanitize=address,undefined
#   etcd_amd/build_san/libetcd_quorum_tsan.so  ... under -fsanitize=thread
#                                              (the std::thread packer)
#   etcd_amd/build_san/liborc_asan.so          the C oracle under ASan+UBSan
# The device code and the other host objects are the main build's
# (etcd_amd/build/*.o): GPU sanitizers are not available on this pool, and
# only host code is instrumented.  Used by tests/test_sanitizers.py, which
# runs the packing and oracle tests against them (LD_PRELOAD of gcc's
# runtimes, since the Python interpreter itself is not instrumented).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/etcd_amd/build_san
mkdir -p "$O"
OBJS=$(ls "$R"/etcd_amd/build/*.o | grep -v '/qe_pack.o$')
for kind in asan tsan; do
  if [ $kind = asan ]; then F="-fsanitize=address,undefined -fno-omit-frame-pointer"; else F="-fsanitize=thread"; fi
  g++ -O1 -g -std=c++17 -fPIC -Wall -Wextra -pthread $F -c -o "$O/qe_pack_$kind.o" "$R/etcd_amd/csrc/qe_pack.cpp"
  g++ -shared -pthread $F -o "$O/libetcd_quorum_$kind.so" $OBJS "$O/qe_pack_$kind.o" \
      -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lrccl
done
gcc -O1 -g -fPIC -fopenmp -Wall -Wextra -std=c11 -D_POSIX_C_SOURCE=199309L \
    -fsanitize=address,undefined -fno-omit-frame-pointer -shared \
    -o "$O/liborc_asan.so" "$R/oracle/quorum_oracle.c"
echo "sanitizer builds in $O"
