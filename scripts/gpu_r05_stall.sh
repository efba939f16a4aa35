#!/bin/bash
# Where a wave's cycles go (r05): SQ_WAVE_CYCLES split into waiting on a
# counter (SQ_WAIT_ANY), waiting for an issue slot (SQ_WAIT_INST_ANY) and
# issuing (SQ_ACTIVE_INST_*), one rocprofv3 --pmc pass per workload.
#   WLS="progress_step config2_n5" bash scripts/gpu_r05_stall.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/stall"; mkdir -p "$O"
for W in ${WLS:-progress_step config2_n5}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$O/$W" -o st -- python3 "$R/bench.py" --workload $W --no-aux --no-cpu-baseline --steps 5 --warmup 1 \
    > "$O/$W.log" 2>&1 || { echo "$W stall pass failed"; tail -5 "$O/$W.log"; exit 3; }
  echo "$W done"
done
