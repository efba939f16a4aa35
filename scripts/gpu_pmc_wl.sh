#!/bin/bash
# PMC passes (one counter group per run) over one bench workload via
# scripts/tune_bench.py; prints per-kernel means for kernels matching $KSUB.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
WL=${WL:-progress_step}; KSUB=${KSUB:-k_progress_step}
O="$R/gpurun_out/pmc_$WL"; rm -rf "$O"; mkdir -p "$O"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  TUNE_WL=$WL TUNE_TPW=-1 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$O/p$i" -o pmc -- python3 "$R/scripts/tune_bench.py" > "$O/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail "$O/p$i.log"; exit 3; }
done
python3 - "$O" "$KSUB" <<'PY'
import csv, glob, sys
agg = {}
for f in sorted(glob.glob(sys.argv[1] + "/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print({k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
