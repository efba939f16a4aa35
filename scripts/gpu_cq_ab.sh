#!/bin/bash
# CheckQuorum parity tests on the built library, then an in-process A/B of
# the main library against the variants under etcd_amd/lib/variants/.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "check_quorum or CheckQuorum or trace" -x -q --timeout 120 --timeout-method thread > gpurun_out/cq_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/cq_tests.log; exit 3; }
tail -2 gpurun_out/cq_tests.log
rm -f gpurun_out/ab_libs.log
WL=check_quorum bash scripts/gpu_ab_libs.sh > /dev/null && WL=check_quorum bash scripts/gpu_ab_libs.sh > /dev/null && WL=check_quorum bash scripts/gpu_ab_libs.sh
