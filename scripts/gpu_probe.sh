#!/bin/bash
# vmem_probe (what a vector memory instruction costs), confchange GPU tests,
# then the confchange workload with and without block-row staging.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 ./scripts/vmem_probe > gpurun_out/vmem_probe.log 2>&1 || { echo probe failed; tail gpurun_out/vmem_probe.log; exit 3; }
cat gpurun_out/vmem_probe.log
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_confchange.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/cc_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ -f gpurun_out/cc_tests.log ] && tail -3 gpurun_out/cc_tests.log
[ $rc -ne 0 ] && exit $rc
TUNE_WL=confchange TUNE_TPW=-1 TUNE_KNOB=cc_block=0,1 timeout -k 10 300 python -u scripts/tune_bench.py 2>&1 | grep -v amdgpu.ids
