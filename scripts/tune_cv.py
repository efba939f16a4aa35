#!/usr/bin/env python3
"""In-process interleaved A/B of launch knobs for qe_commit_vote on the
headline workload (64M groups x 5 voters).  Prints one JSON line per
variant: median / min kernel ms and achieved GB/s (algorithmic bytes).
Library variant chosen with QE_LIB (e.g. a QE_PAIRS=1 build)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from etcd_amd import engine  # noqa: E402

G = int(os.environ.get("TUNE_G", 1 << 26))
S = int(os.environ.get("TUNE_S", 5))
ROUNDS, LAUNCHES = 5, 20
VARIANTS = []
for tpw in [int(x) for x in os.environ.get("TUNE_TPW", "-1,0,1,2,4,8").split(",")]:
    VARIANTS.append({"tiles_per_wave": tpw, "blocks_per_cu": 0, "nontemporal": 3, "stats": 1})
if os.environ.get("TUNE_ONLY_DEFAULT"):
    VARIANTS = VARIANTS[:1]
if os.environ.get("TUNE_VARIANTS"):  # JSON list of knob dicts, e.g. [{"cv_kernel": 1}]
    VARIANTS = [{"stats": 1, **v} for v in json.loads(os.environ["TUNE_VARIANTS"])]
DEFAULTS = {"tiles_per_wave": -1, "blocks_per_cu": 0, "nontemporal": 3, "cv_kernel": -1}
MODE = os.environ.get("TUNE_MODE", "majority")
dev = torch.device("cuda:0")
if MODE == "joint":
    b = engine.SlotBatch(G, S, dev, masks=("inc", "out", "learner"))
    engine.gen_groups(b, 0x5EED, n_inc=S // 2, n_out=S - S // 2,
                      mask_mode=int(os.environ.get("TUNE_MASK_MODE", "0")))
else:
    b = engine.SlotBatch(G, S, dev, masks=())
    engine.gen_groups(b, 0x5EED)
out = engine.Outputs(G, dev, tally=False)
stats = engine.stats_buffer(dev)
gs, os_, os_nostats = b.struct(), out.struct(stats), out.struct(None)
lib = engine._lib.lib()
stream = engine._stream(dev)
bpg = b.bytes_per_group()
res = {i: [] for i in range(len(VARIANTS))}
for r in range(ROUNDS):
    for i, v in enumerate(VARIANTS):
        for k, x in {**DEFAULTS, **v}.items():
            if k != "stats":
                engine.tune(k, x)
        o = os_ if v["stats"] else os_nostats
        for _ in range(3):
            lib.qe_commit_vote(C.byref(gs), C.byref(o), stream)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(LAUNCHES)]
        for a, e in ev:
            a.record()
            lib.qe_commit_vote(C.byref(gs), C.byref(o), stream)
            e.record()
        torch.cuda.synchronize()
        res[i] += [a.elapsed_time(e) for a, e in ev]
for i, v in enumerate(VARIANTS):
    ms = np.array(res[i])
    print(json.dumps({"lib": os.path.basename(engine._lib.LIB_PATH), **v, "S": S, "mode": MODE, "mask_mode": os.environ.get("TUNE_MASK_MODE", "0"),
                      "median_ms": float(np.median(ms)), "min_ms": float(ms.min()),
                      "GBs_median": bpg * G / np.median(ms) / 1e6}))
