#!/bin/bash
# r06: the new GPU tests first (qe_switch_config, the tile-embedded trace
# replays), then the whole GPU suite, then the switch_config workload's bench
# line and its per-workload rocprofv3 passes.  Logs under gpurun_out/$TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
T=${TAG:-r06a}; O=gpurun_out/$T; mkdir -p "$O"
[ "${NEW:-1}" = 1 ] && { timeout -k 10 600 python -u -m pytest tests/test_gpu_switch.py tests/test_gpu_trace_tiles.py tests/test_gpu_readindex.py tests/test_gpu_comm.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/new_tests.log" 2>&1 || { echo "new tests failed"; tail -40 "$O/new_tests.log"; exit 2; }
tail -1 "$O/new_tests.log"; }
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/gpu_tests.log"; exit 3; }
  tail -1 "$O/gpu_tests.log"
fi
for W in ${WLS:-switch_config}; do
  timeout -k 10 300 python -u bench.py --workload $W --no-aux --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -20 "$O/bench_$W.log"; exit 4; }
  tail -1 "$O/bench_$W.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$W', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['bytes_per_unit'])"
done
if [ -n "${AB_WL:-}" ]; then  # in-process A/B of one qe_tune knob (scripts/tune_bench.py)
  TUNE_WL=$AB_WL TUNE_TPW=-1 TUNE_NT=3 TUNE_KNOB=$AB_KNOB timeout -k 10 400 python -u scripts/tune_bench.py \
    > "$O/ab_${AB_WL}.txt" 2>&1 || { echo "A/B failed"; tail -20 "$O/ab_${AB_WL}.txt"; exit 6; }
  cat "$O/ab_${AB_WL}.txt"
fi
if [ "${PROBE:-0}" = 1 ]; then  # the append probe (16-bit ring variants, round 6)
  timeout -k 10 120 ./scripts/append_probe > "$O/append_probe.txt" 2>&1 || { echo "append probe failed"; cat "$O/append_probe.txt"; exit 7; }
  cat "$O/append_probe.txt"
fi
if [ "${PROF:-1}" = 1 ]; then
  WLS="${WLS:-switch_config}" bash scripts/gpu_profile_workloads.sh || exit 5
fi
echo session done
