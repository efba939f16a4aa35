#!/bin/bash
# Progress parity tests on the main library, then scripts/gpu_ab_prog.sh
# (the same tests per variant library, then the interleaved timing).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/abp_main_tests.log 2>&1; rc=$?
echo "main tests rc=$rc"; tail -3 gpurun_out/abp_main_tests.log
[ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab_libs.log
bash scripts/gpu_ab_prog.sh
