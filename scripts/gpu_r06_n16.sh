#!/bin/bash
# r06: the 16-bit Inflights form (ABI 8) -- its GPU differentials, then the
# Progress workloads in both forms on the same (round-6) synthetic state.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
T=${TAG:-r06n}; O=gpurun_out/$T; mkdir -p "$O"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TEST_FILES:-tests/test_gpu_progress.py tests/test_gpu_propose.py tests/test_gpu_switch.py tests/test_gpu_fullsize.py} -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.log"; exit 2; }
  tail -1 "$O/tests.log"
fi
for W in ${WLS:-progress_send propose switch_config progress_step}; do
  for RF in ${FORMS:-0 1}; do
    QE_BENCH_RING16=$RF timeout -k 10 300 python -u bench.py --workload $W --no-aux --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench_${W}_$RF.log" 2>&1 || { echo "bench $W $RF failed"; tail -20 "$O/bench_${W}_$RF.log"; exit 4; }
    tail -1 "$O/bench_${W}_$RF.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$W ring16=$RF', round(d['roofline']['kernel_ms'],4), 'ms frac', round(d['roofline']['frac'],3), 'B/unit', round(d['roofline']['bytes_per_unit'],1))"
  done
done
echo session done
