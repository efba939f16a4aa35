#!/bin/bash
# Round-5 A/B of the pipelined Progress slot loop (QE_PSTEP_PIPE=1 variant,
# scripts/build_variant5.sh pipe "-DQE_PSTEP_PIPE=1"): parity of the variant on
# the S = 5 progress/propose tests with rings in row form (F <= 8), then the
# in-process timing of the main library and the variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=gpurun_out/${TAG:-r05c}; mkdir -p "$O"
V=$R/etcd_amd/lib/variants/libetcd_quorum_pipe.so
QE_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_progress.py tests/test_gpu_trace_replay.py -k "not 32]" \
  > "$O/pipe_tests.log" 2>&1 || { echo "variant parity failed"; tail -30 "$O/pipe_tests.log"; exit 1; }
tail -3 "$O/pipe_tests.log"
WL=${WL:-progress_step,progress_step_joint,config4_repl} bash scripts/gpu_ab_libs.sh
