#!/bin/bash
# bench.py --gpus 2 rehearsal on a 1-GPU box: two ranks spawned by bench.py
# itself (gloo collectives, both ranks on cuda:0), checked against ONE
# process over the union of the two shards (same checksum: the stats
# checksum is an order-free sum keyed by global group id).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
G=${G:-8388608}
export QE_DEVICE_MOD=1 QE_DIST_BACKEND=gloo
timeout -k 10 300 python bench.py --gpus 2 --groups $G --no-aux --no-cpu-baseline --steps 10 --warmup 3 \
  > gpurun_out/rehearse_2ranks.log 2>&1 || { echo "2-rank run failed"; tail -20 gpurun_out/rehearse_2ranks.log; exit 3; }
unset QE_DEVICE_MOD QE_DIST_BACKEND
timeout -k 10 300 python bench.py --gpus 1 --groups $((2*G)) --no-aux --no-cpu-baseline --steps 10 --warmup 3 \
  > gpurun_out/rehearse_union.log 2>&1 || { echo "union run failed"; tail -20 gpurun_out/rehearse_union.log; exit 4; }
python - <<'PY'
import json
a = json.loads([l for l in open("gpurun_out/rehearse_2ranks.log") if l.startswith("{")][-1])
b = json.loads([l for l in open("gpurun_out/rehearse_union.log") if l.startswith("{")][-1])
print("2 ranks: n_gpus", a["n_gpus"], "global_groups", a["config"]["global_groups"], "checksum", a["checks"]["stats_checksum"])
print("union  : n_gpus", b["n_gpus"], "global_groups", b["config"]["global_groups"], "checksum", b["checks"]["stats_checksum"])
assert a["n_gpus"] == 2 and a["config"]["global_groups"] == b["config"]["global_groups"]
assert a["checks"]["stats_checksum"] == b["checks"]["stats_checksum"], "checksum mismatch"
print("REHEARSAL OK")
PY
