#!/bin/bash
# r04 rehearsal of the driver's multi-GPU bench WITH the secondary workloads:
# bench.py --gpus N (N = 4, 8) on a one-GPU box (gloo, every rank on cuda:0),
# each rank at 1/N of every workload's per-GPU size (--groups for the
# headline, --aux-groups-div N for the rest), so the GPU holds about one
# full-size run at a time, as each GPU of the 8-GPU node does.  Records the
# wall time of each run (the driver's timeout budget) and the host packer's
# thread share per rank.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
G=$((1 << 26))
for N in ${NS:-4 8}; do
  t0=$(date +%s.%N)
  QE_DEVICE_MOD=1 QE_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus $N --groups $((G / N)) \
    --aux-groups-div $N --no-cpu-baseline > gpurun_out/reh_aux_$N.log 2>&1 \
    || { echo "$N-rank run failed"; tail -30 gpurun_out/reh_aux_$N.log; exit 3; }
  t1=$(date +%s.%N)
  python3 - "$N" "$t0" "$t1" <<'PY'
import json, sys
n, t0, t1 = int(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3])
d = json.loads([l for l in open(f"gpurun_out/reh_aux_{n}.log") if l.startswith("{")][-1])
print(f"--gpus {n} with aux: wall {t1 - t0:.1f} s, n_gpus {d['n_gpus']}, global groups "
      f"{d['config']['global_groups']}, {len(d['aux'])} aux workloads, invariant violations "
      f"{d['checks']['invariant_violations']}, aux violations "
      f"{sum(v.get('invariant_violations', 0) or 0 for v in d['aux'].values())}")
PY
done
echo rehearsal ok
