#!/bin/bash
# Knob sweep of qe_commit_vote; PAIRS lists extra QE_PAIRS builds to compare.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
LIBS="libetcd_quorum.so"
for p in ${PAIRS:-}; do
  make -s -j16 -C etcd_amd/csrc OBJDIR=../build_p$p LIBOUT=../lib/libetcd_quorum_p$p.so EXTRA=-DQE_PAIRS=$p > gpurun_out/build_p$p.log 2>&1 || { echo build p$p failed; tail gpurun_out/build_p$p.log; exit 2; }
  LIBS="$LIBS libetcd_quorum_p$p.so"
done
rm -f gpurun_out/tune.log
for lib in $LIBS; do
  for cfg in ${CFGS:-majority:5:0 majority:7:0 joint:10:0 joint:10:2}; do
    IFS=: read mode s mm <<< "$cfg"
    QE_LIB=$R/etcd_amd/lib/$lib TUNE_MODE=$mode TUNE_S=$s TUNE_MASK_MODE=$mm TUNE_G=$([ $mode = joint ] && echo 134217728 || echo 67108864) timeout -k 10 240 python scripts/tune_cv.py >> gpurun_out/tune.log 2>&1 || { echo tune failed; tail gpurun_out/tune.log; exit 3; }
  done
done
grep '^{' gpurun_out/tune.log
