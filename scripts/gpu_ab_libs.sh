#!/bin/bash
# In-process timing of bench workloads (scripts/tune_bench.py) with each
# library variant under etcd_amd/lib/variants/ and the main library.
#   WL=progress_step bash scripts/gpu_ab_libs.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; shopt -s nullglob
for L in etcd_amd/lib/libetcd_quorum.so etcd_amd/lib/variants/*.so; do
  QE_LIB=$R/$L TUNE_WL=${WL:-progress_step} TUNE_TPW=${TUNE_TPW:--1} timeout -k 10 300 python -u scripts/tune_bench.py \
    >> gpurun_out/ab_libs.log 2>&1 || { echo "variant $L failed"; tail -5 gpurun_out/ab_libs.log; exit 3; }
done
grep -v amdgpu.ids gpurun_out/ab_libs.log
