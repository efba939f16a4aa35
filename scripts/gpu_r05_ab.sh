#!/bin/bash
# r05 A/B: parity of every variant library under etcd_amd/lib/variants/ on the
# Progress tests (both loop forms: F = 3..32), then the in-process timing of
# the main library and the variants (scripts/gpu_ab_libs.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=gpurun_out/${TAG:-r05h}; mkdir -p "$O"
for L in etcd_amd/lib/variants/*.so; do
  n=$(basename "$L" .so)
  QE_LIB=$R/$L timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_progress.py tests/test_gpu_trace_replay.py ${PTESTS} > "$O/${n}_tests.log" 2>&1 \
    || { echo "$n parity failed"; tail -30 "$O/${n}_tests.log"; exit 1; }
  echo "$n: $(tail -1 "$O/${n}_tests.log")"
done
WL=${WL:-progress_step} bash scripts/gpu_ab_libs.sh
