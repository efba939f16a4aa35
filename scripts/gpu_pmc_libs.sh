#!/bin/bash
# PMC passes (one counter group per run) over one bench workload, for each
# library in $LIBS (A/B of kernel variants); prints per-kernel means of the
# kernels matching $KSUB, one line per library.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
WL=${WL:-progress_step}; KSUB=${KSUB:-k_progress_step}
if [ -n "$SETS_OVERRIDE" ]; then IFS=';' read -ra SETS <<< "$SETS_OVERRIDE"; else
SETS=("FETCH_SIZE" "WRITE_SIZE"
      "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
      "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum"
      "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
      "TD_TD_BUSY_sum TD_TC_STALL_sum"
      "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum")
fi
for L in ${LIBS:-etcd_amd/lib/libetcd_quorum.so}; do
  tag=$(basename "$L" .so)
  O="$R/gpurun_out/pmcl_$tag"; rm -rf "$O"; mkdir -p "$O"
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    QE_LIB="$R/$L" TUNE_WL=$WL TUNE_TPW=-1 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$O/p$i" -o pmc -- python3 "$R/scripts/tune_bench.py" > "$O/p$i.log" 2>&1 || { echo "$tag pmc pass $i failed"; tail "$O/p$i.log"; exit 3; }
  done
  python3 - "$O" "$KSUB" "$tag" <<'PY'
import csv, glob, sys
for ks in sys.argv[2].split(","):
    agg = {}
    for f in sorted(glob.glob(sys.argv[1] + "/p*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if ks not in r["Kernel_Name"]:
                continue
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(sys.argv[3], ks, {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
done
