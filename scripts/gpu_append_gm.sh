#!/bin/bash
# r04: group-major append probe (scripts/append_probe_gm.hip): timing, then
# WRITE_SIZE per kernel (one rocprofv3 pass).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/append_probe_gm > gpurun_out/append_gm.txt 2>&1 || { echo probe failed; cat gpurun_out/append_gm.txt; exit 3; }
cat gpurun_out/append_gm.txt
O=gpurun_out/append_gm_pmc; rm -rf $O
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O -o w -- ./scripts/append_probe_gm > $O.log 2>&1 || { echo pmc failed; tail $O.log; exit 4; }
python3 - $O <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:10s} WRITE_SIZE median {sorted(v)[len(v)//2]/1e3:.1f} MB per launch over {len(v)} launches (KB units x1e3)")
PY
