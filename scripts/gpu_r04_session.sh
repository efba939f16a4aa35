#!/bin/bash
# r04 GPU session: Progress parity on the current library, in-process A/B of
# the Progress workloads against the variants, stamp shares, PMC calibration,
# the append layout probe, then the full bench and Progress kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/prog_tests.log 2>&1 || { echo "progress tests failed"; tail -30 gpurun_out/prog_tests.log; exit 2; }
tail -1 gpurun_out/prog_tests.log
rm -f gpurun_out/ab_libs.log
WL=${ABWL:-progress_step,progress_step_n7,progress_step_joint} bash scripts/gpu_ab_libs.sh || exit 3
if [ -f etcd_amd/lib/variants/libetcd_quorum_stamps.so ] && [ "${STAMPS:-1}" = 1 ]; then
  QE_LIB=$R/etcd_amd/lib/variants/libetcd_quorum_stamps.so TUNE_WL=progress_step,progress_step_n7,progress_step_joint \
    timeout -k 10 240 python scripts/pstep_stamps.py > gpurun_out/stamps.txt 2>&1 || { echo stamps failed; tail gpurun_out/stamps.txt; exit 4; }
  grep -v amdgpu.ids gpurun_out/stamps.txt
fi
[ "${CALIB:-1}" = 1 ] && { bash scripts/gpu_calib.sh || exit 5; bash scripts/gpu_append_gm.sh || exit 6; }
[ "${BENCH:-1}" = 1 ] && { WLS="${KSWLS:-progress_step progress_step_n7 progress_step_joint}" bash scripts/gpu_bench_r04.sh || exit 7; }
echo session done
