#!/bin/bash
# r05 final evidence on one box: the GPU suite (bounded RCCL init first),
# smoke(), the driver's bench command, its rocprofv3 kernel-trace summary,
# and the VALU issue-cost probe with its PMC pass.  Logs under
# gpurun_out/$TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05z}; mkdir -p "$O"
BENCH=0 TAG=${TAG:-r05z} bash scripts/gpu_r05_tests.sh || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; tail -20 "$O/smoke.log"; exit 3; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2>&1 || { echo bench failed; tail -20 "$O/bench.log"; exit 4; }
tail -1 "$O/bench.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('headline', d['value'], d['roofline']['frac'], d['cpu_baseline'] and d['cpu_baseline']['value'])
for k,v in d['aux'].items(): print(f\"{k:24s} {v.get('kernel_ms',0):8.4f} ms  frac {v.get('hbm_frac',0):.3f}\")
"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bench_kt" -o kt -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_kt.log" 2>&1 || { echo "bench kt failed"; tail -20 "$O/bench_kt.log"; exit 5; }
timeout -k 10 120 ./scripts/valu_probe > "$O/valu_probe.txt" 2>&1 || { echo valu probe failed; cat "$O/valu_probe.txt"; exit 6; }
cat "$O/valu_probe.txt"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/valu_pmc" -o v -- ./scripts/valu_probe > "$O/valu_pmc.log" 2>&1 || { echo valu pmc failed; tail "$O/valu_pmc.log"; exit 7; }
for W in config5_elec config5_prevote_cq; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/valu_$W" -o v -- python3 bench.py --workload $W --no-aux --no-cpu-baseline --steps 5 --warmup 1 > "$O/valu_$W.log" 2>&1 || { echo "valu pmc $W failed"; tail "$O/valu_$W.log"; exit 8; }
done
echo session done
