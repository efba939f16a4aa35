#!/bin/bash
# Progress-step parity tests with each variant library, then interleaved
# timing of the progress_step workload for the main library and the variants.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for L in etcd_amd/lib/variants/*.so; do
  QE_LIB=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/abp_tests.log 2>&1; rc=$?
  echo "$L tests rc=$rc"; tail -2 gpurun_out/abp_tests.log
  [ $rc -ne 0 ] && exit $rc
done
WL=${WL:-progress_step} bash scripts/gpu_ab_libs.sh
