#!/bin/bash
# r05: fresh per-workload rocprofv3 passes for the workloads whose committed
# PMC predates this round's code, then the VALU probe (3-source kinds on
# distinct registers) with its PMC pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05x}; mkdir -p "$O"
# the pipelined propose kernel: its parity tests and bench line first
timeout -k 10 600 python -u -m pytest tests/test_gpu_propose.py tests/test_gpu_trace_replay.py tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.log"; exit 5; }
tail -1 "$O/tests.log"
timeout -k 10 300 python -u bench.py --workload propose --no-aux --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench_propose.log" 2>&1 || { echo bench failed; tail -20 "$O/bench_propose.log"; exit 6; }
tail -1 "$O/bench_propose.log" | cut -c1-300
WLS=${WLS:-"config5_elec config5_prevote_cq progress_send propose progress_step_n7"} bash scripts/gpu_profile_workloads.sh || exit 2
timeout -k 10 120 ./scripts/valu_probe > "$O/valu_probe.txt" 2>&1 || { echo valu probe failed; cat "$O/valu_probe.txt"; exit 3; }
cat "$O/valu_probe.txt"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/valu_pmc" -o v -- ./scripts/valu_probe > "$O/valu_pmc.log" 2>&1 || { echo valu pmc failed; tail "$O/valu_pmc.log"; exit 4; }
echo session done
