#!/bin/bash
# SQ/GRBM counters for the commit_vote kernels (majority S=5, joint S=10).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/pmc_sq
export TMPDIR=/tmp
for cfg in majority:5:0 joint:10:2 joint:10:0; do
  IFS=: read mode s mm <<< "$cfg"
  G=$([ $mode = joint ] && echo 134217728 || echo 67108864)
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -c1-12 | tr ' ' '_')
    TUNE_TPW=-1 TUNE_MODE=$mode TUNE_S=$s TUNE_MASK_MODE=$mm TUNE_G=$G timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/pmc_sq/${mode}_${s}_${mm}_$tag" -o pmc -- python3 "$R/scripts/tune_cv.py" > "$R/gpurun_out/pmc_sq/${mode}_${s}_${mm}_$tag.log" 2>&1 || { echo "pmc $cfg failed"; tail "$R/gpurun_out/pmc_sq/${mode}_${s}_${mm}_$tag.log"; exit 3; }
  done
done
python3 - <<'PY'
import csv, glob, os
for f in sorted(glob.glob("gpurun_out/pmc_sq/*/pmc_counter_collection.csv")):
    agg = {}
    for r in csv.DictReader(open(f)):
        if "k_commit_vote" not in r["Kernel_Name"] and "k_cv_stream" not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
