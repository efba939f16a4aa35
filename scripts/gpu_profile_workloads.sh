#!/bin/bash
# Per-workload rocprofv3 evidence: for each bench workload, in runs of its
# own (so no two workloads' launches are averaged together):
#   kt     --kernel-trace --stats (average kernel durations)
#   fetch  --pmc FETCH_SIZE
#   write  --pmc WRITE_SIZE
#   sq     --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
#                SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
#   vmem   --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM
#                SQ_INSTS_VALU_INT64 (vector-memory instruction counts)
#   stall  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_*
#                (where a wave's cycles go; round 5's gpu_r05_stall.sh set)
# PASSES selects the passes (default: all).
# Output: gpurun_out/profw/<workload>/<pass>/...; fold with
#   python scripts/summarize_workloads.py <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
WLS=${WLS:-"config2_n5 config2_n7 config3_joint config3_joint_rot config4_repl config4_repl_joint config5_elec config5_prevote_cq progress_step confchange"}
O="$R/gpurun_out/profw"; mkdir -p "$O"
for W in $WLS; do
  mkdir -p "$O/$W"
  P=" ${PASSES:-kt fetch write sq vmem stall} "
  BA="--workload $W --no-aux --no-cpu-baseline"
  [[ $P == *" kt "* ]] && { timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$W/kt" -o kt -- python3 "$R/bench.py" $BA --steps 20 --warmup 5 > "$O/$W/kt.log" 2>&1 || { echo "$W kt failed"; tail -5 "$O/$W/kt.log"; exit 3; }; }
  [[ $P == *" fetch "* ]] && { timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/$W/fetch" -o fetch -- python3 "$R/bench.py" $BA --steps 5 --warmup 1 > "$O/$W/fetch.log" 2>&1 || { echo "$W fetch failed"; tail -5 "$O/$W/fetch.log"; exit 4; }; }
  [[ $P == *" write "* ]] && { timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/$W/write" -o write -- python3 "$R/bench.py" $BA --steps 5 --warmup 1 > "$O/$W/write.log" 2>&1 || { echo "$W write failed"; tail -5 "$O/$W/write.log"; exit 5; }; }
  [[ $P == *" sq "* ]] && { timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$O/$W/sq" -o sq -- python3 "$R/bench.py" $BA --steps 5 --warmup 1 > "$O/$W/sq.log" 2>&1 || { echo "$W sq failed"; tail -5 "$O/$W/sq.log"; exit 6; }; }
  [[ $P == *" vmem "* ]] && { timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_INT64 --output-format csv -d "$O/$W/vmem" -o vmem -- python3 "$R/bench.py" $BA --steps 5 --warmup 1 > "$O/$W/vmem.log" 2>&1 || { echo "$W vmem failed"; tail -5 "$O/$W/vmem.log"; exit 7; }; }
  [[ $P == *" stall "* ]] && { timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d "$O/$W/stall" -o stall -- python3 "$R/bench.py" $BA --steps 5 --warmup 1 > "$O/$W/stall.log" 2>&1 || { echo "$W stall failed"; tail -5 "$O/$W/stall.log"; exit 8; }; }
  echo "$W done"
done
