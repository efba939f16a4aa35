#!/bin/bash
# r04: one full default bench.py run (headline + every aux workload), then
# per-kernel average durations (rocprofv3 --kernel-trace --stats) of the
# Progress workloads (WLS) through scripts/tune_bench.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 3; }
  tail -1 gpurun_out/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('headline', d['value'], d['roofline']['frac'])
for k,v in d['aux'].items(): print(f\"{k:24s} {v.get('kernel_ms',0):8.4f} ms  frac {v.get('hbm_frac',0):.3f}\")
print('cpu', {k: d['cpu_baseline'][k] for k in ('value','cores','one_thread_value','full_host_value')} if d.get('cpu_baseline') else None)
"
fi
for WL in ${WLS:-}; do
  O="$R/gpurun_out/kstats_$WL"; rm -rf "$O"; mkdir -p "$O"
  TUNE_WL=$WL TUNE_TPW=-1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o ks -- python3 "$R/scripts/tune_bench.py" > "$O/run.log" 2>&1 || { echo "kstats $WL failed"; tail "$O/run.log"; exit 4; }
  grep -h "median" "$O/run.log"
  python3 - "$O" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs'])/1e3:10.1f} us  x{r['Calls']:>5}  {r['Name'][:110]}")
PY
done
echo done
