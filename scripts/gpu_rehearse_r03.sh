#!/bin/bash
# r03: bench.py --gpus 4 and --gpus 8 rehearsals on a 1-GPU box (gloo, every
# rank on cuda:0, 2M groups per rank) against one process over the union of
# the shards, for the headline and the Progress-step workload (state keyed by
# global group id): the aggregated checksum must be identical.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
G=2097152
for WL in config2_n5 progress_step; do
  for N in 4 8; do
    QE_DEVICE_MOD=1 QE_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus $N --groups $G \
      --workload $WL --no-aux --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/reh_${WL}_$N.log 2>&1 \
      || { echo "$WL $N-rank run failed"; tail -20 gpurun_out/reh_${WL}_$N.log; exit 3; }
    timeout -k 10 300 python bench.py --gpus 1 --groups $((N*G)) --workload $WL --no-aux \
      --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/reh_${WL}_union$N.log 2>&1 \
      || { echo "$WL union $N failed"; tail -20 gpurun_out/reh_${WL}_union$N.log; exit 4; }
    python - "$WL" "$N" <<'PY'
import json, sys
wl, n = sys.argv[1], sys.argv[2]
a = json.loads([l for l in open(f"gpurun_out/reh_{wl}_{n}.log") if l.startswith("{")][-1])
b = json.loads([l for l in open(f"gpurun_out/reh_{wl}_union{n}.log") if l.startswith("{")][-1])
print(wl, n, "ranks: n_gpus", a["n_gpus"], "global", a["config"]["global_groups"], "checksum",
      a["checks"]["stats_checksum"], "| union: global", b["config"]["global_groups"], "checksum",
      b["checks"]["stats_checksum"])
assert a["n_gpus"] == int(n) and a["config"]["global_groups"] == b["config"]["global_groups"]
assert a["checks"]["stats_checksum"] == b["checks"]["stats_checksum"]
PY
    [ $? -eq 0 ] || exit 5
  done
done
echo rehearsal ok
