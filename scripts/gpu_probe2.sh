#!/bin/bash
# tlb_probe, then config4_repl with the full-row variant vs the main library.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 ./scripts/tlb_probe > gpurun_out/tlb_probe.log 2>&1 || { echo probe failed; tail gpurun_out/tlb_probe.log; exit 3; }
cat gpurun_out/tlb_probe.log
exit 0
  --timeout 120 --timeout-method thread > gpurun_out/p2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/p2_tests.log
[ $rc -ne 0 ] && exit $rc
QE_LIB=$R/etcd_amd/lib/variants/libetcd_quorum_replfull.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "repl or replication" -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/p2_tests_v.log 2>&1; rc=$?
echo "variant tests rc=$rc"; tail -2 gpurun_out/p2_tests_v.log
[ $rc -ne 0 ] && exit $rc
WL=config4_repl bash scripts/gpu_ab_libs.sh
