#!/bin/bash
# Round-5 A/B of the pipelined Progress slot loop (variants of the S = 5, 6, 7
# objects: OBJS="qe_inst_prog_5 qe_inst_prog_6 qe_inst_prog_7"
# scripts/build_variant5.sh pipe "-DQE_PSTEP_PIPE=1", and pipe2 with
# -DQE_PSTEP_PIPE=2): parity of each variant on the Progress tests (pipe: rings
# in row form only, F <= 8; pipe2: every test), then the in-process timing of
# the main library and the variants.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=gpurun_out/${TAG:-r05c}; mkdir -p "$O"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
if [ -f etcd_amd/lib/variants/libetcd_quorum_pipe.so ]; then
  QE_LIB=$R/etcd_amd/lib/variants/libetcd_quorum_pipe.so timeout -k 10 600 $T \
    tests/test_gpu_progress.py tests/test_gpu_trace_replay.py -k "not 32] and not long_rings" \
    > "$O/pipe_tests.log" 2>&1 || { echo "pipe parity failed"; tail -30 "$O/pipe_tests.log"; exit 1; }
  tail -1 "$O/pipe_tests.log"
fi
if [ -f etcd_amd/lib/variants/libetcd_quorum_pipe2.so ]; then
  QE_LIB=$R/etcd_amd/lib/variants/libetcd_quorum_pipe2.so timeout -k 10 600 $T \
    tests/test_gpu_progress.py tests/test_gpu_trace_replay.py tests/test_gpu_propose.py \
    > "$O/pipe2_tests.log" 2>&1 || { echo "pipe2 parity failed"; tail -30 "$O/pipe2_tests.log"; exit 1; }
  tail -1 "$O/pipe2_tests.log"
fi
WL=${WL:-progress_step,progress_step_n7,progress_step_joint} bash scripts/gpu_ab_libs.sh
