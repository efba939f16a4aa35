#!/bin/bash
# Round-3 full pass: GPU tests, smoke, default bench (N=1, all aux), and the
# headline's kernel trace.  Each GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -6 gpurun_out/gpu_tests.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 3; }
  tail -1 gpurun_out/smoke.log
fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
grep "^{" gpurun_out/bench.log | tail -1 | cut -c1-600
if [ "${SKIP_KT:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-aux > gpurun_out/kt.log 2>&1 || { echo ktrace failed; tail -5 gpurun_out/kt.log; exit 5; }
  find gpurun_out/kt -name "*stats*.csv" | head
fi
echo done
