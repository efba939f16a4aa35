#!/bin/bash
# Heartbeat tiles-per-wave sweep on the main library (in-process, tune_bench).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for i in 1 2; do
TUNE_WL=heartbeat TUNE_TPW=-1,1,2,4,8 timeout -k 10 300 python -u scripts/tune_bench.py >> gpurun_out/hb_tpw.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/hb_tpw.log; exit 3; }
done
grep -v amdgpu gpurun_out/hb_tpw.log
