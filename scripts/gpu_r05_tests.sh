#!/bin/bash
# r05: the GPU test suite (comm tests first: the bounded RCCL init), then
# optionally one default bench.py run.  Logs under gpurun_out/$TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05}; mkdir -p "$O"
timeout -k 10 200 python -u -m pytest tests/test_gpu_comm.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$O/comm_tests.log" 2>&1 || { echo "comm tests failed"; tail -30 "$O/comm_tests.log"; exit 2; }
tail -1 "$O/comm_tests.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} \
  --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/gpu_tests.log"; exit 3; }
tail -2 "$O/gpu_tests.log"
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1 || { echo bench failed; tail -20 "$O/bench.log"; exit 4; }
  tail -1 "$O/bench.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('headline', d['value'], d['roofline']['frac'])
for k,v in d['aux'].items(): print(f\"{k:24s} {v.get('kernel_ms',0):8.4f} ms  frac {v.get('hbm_frac',0):.3f}\")
"
fi
echo session done
