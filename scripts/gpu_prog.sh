#!/bin/bash
# Progress-step kernel on the GPU box: parity tests, then an interleaved
# in-process timing of library variants (scripts/tune_bench.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/prog_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ -n "$NOTEST" ] || tail -5 gpurun_out/prog_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/prog_tune.log
for L in ${LIBS:-etcd_amd/lib/libetcd_quorum.so}; do
  QE_LIB="$R/$L" TUNE_WL=${TUNE_WL:-progress_step} TUNE_TPW=${TUNE_TPW:--1} \
    timeout -k 10 300 python -u scripts/tune_bench.py >> gpurun_out/prog_tune.log 2>&1 || { echo "tune $L failed"; tail gpurun_out/prog_tune.log; exit 5; }
done
grep -v amdgpu.ids gpurun_out/prog_tune.log
