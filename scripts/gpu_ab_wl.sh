#!/bin/bash
# Interleaved timing of bench workloads ($WL, comma list) for the main
# library and each variant under etcd_amd/lib/variants/ (TUNE_TPW knob list).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; shopt -s nullglob
for L in etcd_amd/lib/libetcd_quorum.so etcd_amd/lib/variants/*.so; do
  QE_LIB=$R/$L TUNE_WL=$WL TUNE_TPW=${TUNE_TPW:--1} timeout -k 10 400 python -u scripts/tune_bench.py \
    >> gpurun_out/ab_wl.log 2>&1 || { echo "variant $L failed"; tail -5 gpurun_out/ab_wl.log; exit 3; }
done
grep -v amdgpu.ids gpurun_out/ab_wl.log
