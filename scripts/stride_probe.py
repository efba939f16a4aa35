#!/usr/bin/env python3
"""Slot-row spacing A/B (round 6).  The slot-SoA rows of a ProgressState are
`stride` groups apart; at the bench's G = 2^24 that is a power of two
(128 MiB between Match rows, 512 MiB between ring rows), so the S rows a
tile touches, and every per-slot array, start at the same offset modulo
any power of two.  This runs bench workloads with stride = G + PAD groups.

  PAD=0 WLS=progress_send,switch_config python scripts/stride_probe.py

One process per PAD value (a workload's time also depends on what ran
before it in the process: scripts/order_probe.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from etcd_amd import engine  # noqa: E402

bench.engine = engine
PAD = int(os.environ.get("PAD", "0"))
_PS = engine.ProgressState


class PaddedState(_PS):
    def __init__(self, G, S, F, R, *a, stride=None, **k):
        st = stride or (-(-int(G) // 64) * 64 + PAD)
        super().__init__(G, S, F, R, *a, stride=st, **k)


engine.ProgressState = PaddedState


def main():
    args = bench.parse([])
    args.workload = "config2_n5"
    d = bench.Dist()
    for name in os.environ.get("WLS", "progress_send").split(","):
        r = bench.run_workload(name, args, d, 20, 5)
        print(f"pad {PAD:6d} {name:20s} kernel {r['kernel_ms']:.4f} ms  frac {r['hbm_frac']:.3f}"
              f"  checksum {r['checksum']}", flush=True)


if __name__ == "__main__":
    main()
