#!/bin/bash
# GPU parity tests, then in-process timing of the named bench workloads
# (scripts/tune_bench.py).  WL=comma list, TESTS=pytest paths, K=-k expression.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && exit $rc
TUNE_WL=${WL:-config3_joint} TUNE_TPW=${TUNE_TPW:--1} timeout -k 10 400 python -u scripts/tune_bench.py > gpurun_out/quick_tune.log 2>&1 || { echo tune failed; tail gpurun_out/quick_tune.log; exit 5; }
grep -v amdgpu.ids gpurun_out/quick_tune.log
