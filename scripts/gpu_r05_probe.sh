#!/bin/bash
# r05: the Progress/leader-round scenarios on the GPU, then the VALU
# issue-cost probe (all its kinds) and its PMC pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05y}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_progress.py -m gpu -x -q -p no:cacheprovider -k "scenarios" \
  --timeout 120 --timeout-method thread > "$O/scen_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/scen_tests.log"; exit 2; }
tail -1 "$O/scen_tests.log"
timeout -k 10 120 ./scripts/valu_probe > "$O/valu_probe.txt" 2>&1 || { echo valu probe failed; cat "$O/valu_probe.txt"; exit 3; }
cat "$O/valu_probe.txt"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/valu_pmc" -o v -- ./scripts/valu_probe > "$O/valu_pmc.log" 2>&1 || { echo valu pmc failed; tail "$O/valu_pmc.log"; exit 4; }
echo session done
