#!/bin/bash
# A/B of qe_commit_vote kernels on the GPU box: parity subset first, then
# interleaved in-process timing (scripts/tune_cv.py) per workload.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/ab_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -5 gpurun_out/ab_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
V=${VARIANTS:-'[{"cv_kernel":0},{"cv_kernel":1}]'}
: > gpurun_out/ab.jsonl
WL=${WORKLOADS:-"joint:10:2 joint:10:0 majority:5:0 majority:7:0"}
LIBS=${LIBS:-etcd_amd/lib/libetcd_quorum.so}
for L in $LIBS; do
for W in $WL; do
  IFS=: read M S MM <<< "$W"
  G=$((1<<26)); [ "$M" = joint ] && G=$((1<<27))
  QE_LIB="$R/$L" TUNE_MODE=$M TUNE_S=$S TUNE_MASK_MODE=$MM TUNE_G=$G TUNE_VARIANTS="$V" \
    timeout -k 10 300 python -u scripts/tune_cv.py >> gpurun_out/ab.jsonl 2> gpurun_out/ab_err.log || { echo "tune $W failed"; tail gpurun_out/ab_err.log; exit 5; }
done
done
cat gpurun_out/ab.jsonl
if [ -n "${BENCH_WL:-}" ]; then
  timeout -k 10 300 python bench.py --workload "$BENCH_WL" --no-aux --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ab_bench.log 2>&1 || { echo bench failed; tail gpurun_out/ab_bench.log; exit 6; }
  tail -1 gpurun_out/ab_bench.log
fi
