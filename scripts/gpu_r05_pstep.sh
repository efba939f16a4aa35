#!/bin/bash
# r05: the pipelined Progress slot loop in the product library -- the whole
# GPU suite, the Progress bench workloads, then their rocprofv3 passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05f}; mkdir -p "$O"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -40 "$O/gpu_tests.log"; exit 2; }
  tail -2 "$O/gpu_tests.log"
fi
for W in ${BWLS:-progress_step progress_step_n7 progress_step_joint}; do
  timeout -k 10 300 python -u bench.py --workload $W --no-aux --no-cpu-baseline --steps 20 --warmup 5 > "$O/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -20 "$O/bench_$W.log"; exit 3; }
  tail -1 "$O/bench_$W.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$W', d['value'], r['kernel_ms'], r['frac'])"
done
WLS=${WLS:-"progress_step progress_step_n7 progress_step_joint"} bash scripts/gpu_profile_workloads.sh || exit 4
echo session done
