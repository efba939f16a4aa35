#!/bin/bash
# Knob sweep of qe_commit_vote.  BUILDS="name:-DFLAG=V ..." adds library
# variants compiled on the box; CFGS="mode:S:mask_mode ..." picks workloads.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
LIBS="libetcd_quorum.so"
for b in ${BUILDS:-}; do
  name=${b%%:*}; flags=${b#*:}
  make -s -j16 -C etcd_amd/csrc OBJDIR=../build_$name LIBOUT=../lib/libetcd_quorum_$name.so "EXTRA=$flags" > gpurun_out/build_$name.log 2>&1 || { echo build $name failed; tail gpurun_out/build_$name.log; exit 2; }
  LIBS="$LIBS libetcd_quorum_$name.so"
done
rm -f gpurun_out/tune.log
for lib in $LIBS; do
  for cfg in ${CFGS:-majority:5:0 majority:7:0 joint:10:0 joint:10:2}; do
    IFS=: read mode s mm <<< "$cfg"
    QE_LIB=$R/etcd_amd/lib/$lib TUNE_MODE=$mode TUNE_S=$s TUNE_MASK_MODE=$mm TUNE_G=$([ $mode = joint ] && echo 134217728 || echo 67108864) timeout -k 10 240 python scripts/tune_cv.py >> gpurun_out/tune.log 2>&1 || { echo tune failed; tail gpurun_out/tune.log; exit 3; }
  done
done
grep '^{' gpurun_out/tune.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'][15:], d['mode'], d['S'], d['mask_mode'], 'tpw', d['tiles_per_wave'], 'nt', d['nontemporal'], 'med %.4f min %.4f' % (d['median_ms'], d['min_ms']))
"
