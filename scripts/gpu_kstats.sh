#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of one
# bench workload run through scripts/tune_bench.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
WL=${WL:-progress_step}
O="$R/gpurun_out/kstats_$WL"; rm -rf "$O"; mkdir -p "$O"
TUNE_WL=$WL TUNE_TPW=${TUNE_TPW:--1} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o ks -- python3 "$R/scripts/tune_bench.py" > "$O/run.log" 2>&1 || { echo "kstats failed"; tail "$O/run.log"; exit 3; }
python3 - "$O" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs'])/1e3:10.1f} us  x{r['Calls']:>5}  {r['Name'][:110]}")
PY
