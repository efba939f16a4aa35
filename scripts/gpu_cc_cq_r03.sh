#!/bin/bash
# r03: confchange / check_quorum pipeline rewrite -- GPU tests of both entry
# points, then an in-process A/B against the previous library (variants/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_confchange.py tests/test_gpu_progress.py > gpurun_out/cc_cq_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cc_cq_tests.log; [ $rc -eq 0 ] || exit $rc
WL=confchange,check_quorum bash scripts/gpu_ab_libs.sh
