#!/bin/bash
# (1) HBM ceiling probe; (2) 2-rank rehearsal of bench.py's multi-process path
# on a 1-GPU box (gloo for the collectives, both ranks on cuda:0).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/membw scripts/membw.hip || exit 2
timeout -k 10 120 /tmp/membw > gpurun_out/membw.log 2>&1 || { echo membw failed; cat gpurun_out/membw.log; exit 3; }
cat gpurun_out/membw.log
QE_DIST_BACKEND=gloo QE_DEVICE_MOD=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --no-aux > gpurun_out/rehearse2.log 2>&1 || { echo rehearsal failed; tail -20 gpurun_out/rehearse2.log; exit 4; }
grep '^{' gpurun_out/rehearse2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n_gpus', d['n_gpus'], 'value', d['value'], 'global_groups', d['config']['global_groups'], 'checks', d['checks'], 'cpu', d['cpu_baseline'])"
