#!/bin/bash
# confchange on the GPU box: parity tests, then interleaved timing of the
# confchange bench workload for each library in $LIBS.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_confchange.py tests/test_cpp_api.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/cc_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/cc_tests.log
[ $rc -ne 0 ] && exit $rc
for L in ${LIBS:-etcd_amd/lib/libetcd_quorum.so}; do
  QE_LIB="$R/$L" TUNE_WL=confchange TUNE_TPW=-1 timeout -k 10 300 python -u scripts/tune_bench.py 2>&1 | grep -v amdgpu.ids || exit 5
done
