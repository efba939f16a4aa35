#!/bin/bash
# r03: ABI 4 rings (32-bit words, lane-major, epoch / wide form) -- Progress
# GPU tests, then in-process timing of the Progress workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_progress.py tests/test_gpu_confchange.py > gpurun_out/ring32_tests.log 2>&1
rc=$?; tail -5 gpurun_out/ring32_tests.log; [ $rc -eq 0 ] || exit $rc
TUNE_WL=${WL:-progress_step,progress_send,check_quorum} TUNE_TPW=-1 timeout -k 10 300 \
  python -u scripts/tune_bench.py > gpurun_out/ring32_tune.log 2>&1 || { tail -5 gpurun_out/ring32_tune.log; exit 4; }
grep -v amdgpu.ids gpurun_out/ring32_tune.log
