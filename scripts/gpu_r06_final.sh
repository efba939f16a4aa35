#!/bin/bash
# r06 evidence on one box: the GPU suite (bounded RCCL init first), smoke(),
# the driver's bench command, its rocprofv3 kernel-trace summary, then the
# per-workload rocprofv3 passes of $WLS on the same box (kernel trace, FETCH,
# WRITE, SQ, vmem, stall), so a workload's rocprof average and its bench
# line come from one machine.  Logs under gpurun_out/$TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
T=${TAG:-r06f}; O=gpurun_out/$T; mkdir -p "$O"
if [ "${TESTS:-1}" = 1 ]; then
  BENCH=0 TAG=$T bash scripts/gpu_r05_tests.sh || exit 2
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; tail -20 "$O/smoke.log"; exit 3; }
  tail -1 "$O/smoke.log"
fi
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2>&1 || { echo bench failed; tail -20 "$O/bench.log"; exit 4; }
tail -1 "$O/bench.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('headline', d['value'], d['roofline']['frac'], d['cpu_baseline'] and d['cpu_baseline']['value'])
for k,v in d['aux'].items(): print(f\"{k:24s} {v.get('kernel_ms',0):8.4f} ms  frac {v.get('hbm_frac',0):.3f}\")
"
if [ "${KT:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bench_kt" -o kt -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_kt.log" 2>&1 || { echo "bench kt failed"; tail -20 "$O/bench_kt.log"; exit 5; }
fi
if [ -n "${WLS:-}" ]; then
  WLS="$WLS" bash scripts/gpu_profile_workloads.sh || exit 6
fi
echo session done
