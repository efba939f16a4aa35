#!/bin/bash
# r05: qe_propose on the GPU -- its tests and the Progress tests that now
# append through it, the bench workload, then its rocprofv3 passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05b}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_propose.py tests/test_gpu_trace_replay.py tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.log"; exit 2; }
tail -2 "$O/tests.log"
timeout -k 10 300 python -u bench.py --workload propose --no-aux --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench_propose.log" 2>&1 || { echo bench failed; tail -20 "$O/bench_propose.log"; exit 3; }
tail -1 "$O/bench_propose.log" | cut -c1-600
WLS=${WLS:-propose} bash scripts/gpu_profile_workloads.sh || exit 4
# VALU issue cost per instruction kind, and what the SQ counters report for it
timeout -k 10 120 ./scripts/valu_probe > "$O/valu_probe.txt" 2>&1 || { echo valu probe failed; cat "$O/valu_probe.txt"; exit 5; }
cat "$O/valu_probe.txt"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/valu_pmc" -o v -- ./scripts/valu_probe > "$O/valu_pmc.log" 2>&1 || { echo valu pmc failed; tail "$O/valu_pmc.log"; exit 6; }
for W in config5_elec config5_prevote_cq; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/valu_$W" -o v -- python3 bench.py --workload $W --no-aux --no-cpu-baseline --steps 5 --warmup 1 > "$O/valu_$W.log" 2>&1 || { echo "valu pmc $W failed"; tail "$O/valu_$W.log"; exit 7; }
done
echo session done
