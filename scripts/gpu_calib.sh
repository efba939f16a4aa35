#!/bin/bash
# r04: FETCH_SIZE / WRITE_SIZE calibration by access width (scripts/pmc_calib.hip).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/calib; rm -rf $O; mkdir -p $O
timeout -k 10 120 ./scripts/pmc_calib > $O/probe.txt 2>&1 || { echo calib probe failed; cat $O/probe.txt; exit 3; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o f -- ./scripts/pmc_calib > $O/fetch.log 2>&1 || { echo fetch pass failed; tail $O/fetch.log; exit 4; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o w -- ./scripts/pmc_calib > $O/write.log 2>&1 || { echo write pass failed; tail $O/write.log; exit 5; }
python3 scripts/pmc_calib.py $O/probe.txt $O/fetch $O/write $O/calib.json
