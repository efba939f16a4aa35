#!/usr/bin/env python3
"""Section shares of the Progress step's wave cycles from the stamp build
(QE_PSTEP_STAMPS, scripts/build_variant5.sh): one bench
workload, LAUNCHES launches, the per-section sums of s_memtime deltas
(100 MHz ticks) over all waves, printed as shares.

  QE_LIB=etcd_amd/lib/variants/libetcd_quorum_stamps.so TUNE_WL=progress_step python scripts/pstep_stamps.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from etcd_amd import engine  # noqa: E402

bench.engine = engine
NAMES = ["tile head: round trips 1-2 + phase 1", "slot: loads (Progress, ring, runs)",
         "bcasts before the message (k1 burst)", "message handler", "the message's sends + loop + later bcasts",
         "ring write-back", "Progress stores + outputs", "tile tail (group outputs)"]


def main():
    d = bench.Dist()
    for wl in os.environ.get("TUNE_WL", "progress_step").split(","):
        desc, G, S, kind = bench.WORKLOADS[wl]
        stats = engine.stats_buffer(d.dev)
        step, bpu, units, _, keep = bench.setup(wl, G, S, kind, d, stats)
        msgs, prep = keep["msgs"], keep["prepare"]
        acc = torch.zeros(16, dtype=torch.int64, device=d.dev)
        msgs.bytes_requested = acc
        for _ in range(3):
            prep()
            engine.progress_step(keep["ps"], msgs)
        acc.zero_()
        n = int(os.environ.get("LAUNCHES", "10"))
        for _ in range(n):
            prep()
            engine.progress_step(keep["ps"], msgs)
        torch.cuda.synchronize()
        v = acc.cpu().numpy()
        tot = float(v[:8].sum())
        print(f"{wl}: {int(v[8]) // n} tiles per launch, {tot / max(1, v[8]):.0f} s_memtime ticks per tile")
        for k, name in enumerate(NAMES):
            print(f"  {v[k] / tot:6.3f}  {name}")
        del keep
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
