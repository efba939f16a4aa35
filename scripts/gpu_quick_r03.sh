#!/bin/bash
# Focused GPU pass: selected tests, then selected bench workloads (no aux).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -15 gpurun_out/quick_tests.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for w in ${WORKLOADS:-}; do
  timeout -k 10 300 python -u bench.py --workload $w --no-aux --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 > gpurun_out/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 gpurun_out/bench_$w.log; exit 4; }
  python - "$w" <<'PY'
import json, sys
w = sys.argv[1]
line = [l for l in open(f"gpurun_out/bench_{w}.log") if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print(f"{w}: value={d['value']:.4g} {d['unit']} kernel_ms={r['kernel_ms']:.4f} bpu={r['bytes_per_unit']:.1f} frac={r['frac']:.3f}")
PY
done
