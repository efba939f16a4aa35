#!/bin/bash
# Parity tests (TESTS, -k KSEL) then an in-process A/B of one qe_tune knob
# over bench workloads (scripts/tune_bench.py), each step under its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider ${KSEL:+-k "$KSEL"} \
    --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -5 gpurun_out/ab_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
TUNE_WL=${TUNE_WL:-config4_repl} TUNE_TPW=${TUNE_TPW:--1} TUNE_KNOB=${TUNE_KNOB:-} \
  timeout -k 10 400 python -u scripts/tune_bench.py > gpurun_out/ab_tune.log 2>&1 || { echo tune failed; tail gpurun_out/ab_tune.log; exit 5; }
grep -v amdgpu.ids gpurun_out/ab_tune.log
