#!/bin/bash
# 2-rank rehearsal of the driver's multi-GPU bench (aux workloads included)
# on a 1-GPU box: both ranks on cuda:0, gloo for the collectives.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
QE_DIST_BACKEND=gloo QE_DEVICE_MOD=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/rehearse2_aux.log 2>&1 || { echo rehearsal failed; tail -30 gpurun_out/rehearse2_aux.log; exit 4; }
grep '^{' gpurun_out/rehearse2_aux.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n_gpus', d['n_gpus'], 'value', d['value'], {k: round(v['value']/1e9,2) for k,v in d['aux'].items()})"
