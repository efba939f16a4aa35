#!/bin/bash
# GPU parity tests, one process, per-test time limit; then smoke.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -40
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
