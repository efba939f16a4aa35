#!/usr/bin/env python3
"""Array placement A/B (round 6): the Progress arrays of a ProgressState
as views of ONE device allocation (a slab), each array starting at a 2 MiB
boundary plus SKEW * its index bytes, against the default (one allocation per
array, placed by the allocator).  scripts/order_probe.py showed the
scatter-heavy kernels (progress_send, switch_config, propose) 7-20 % faster
or slower depending on what the process allocated before -- with the same
state (equal checksums).  This asks whether a fixed placement removes that.

  SLAB=1 SKEW=0 WLS=progress_send,switch_config python scripts/slab_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from etcd_amd import engine  # noqa: E402

bench.engine = engine
SLAB = os.environ.get("SLAB", "1") == "1"
SKEW = int(os.environ.get("SKEW", "0"))
_PS = engine.ProgressState


class SlabState(_PS):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        if not SLAB:
            return
        names = [n for n in self.ARRAYS if getattr(self, n, None) is not None]
        offs, off = {}, 0
        for i, n in enumerate(names):
            off = -(-off // (2 << 20)) * (2 << 20) + SKEW * i
            offs[n] = off
            off += getattr(self, n).numel() * getattr(self, n).element_size()
        slab = torch.empty(off, dtype=torch.uint8, device=self.device)
        for n in names:
            t = getattr(self, n)
            nb = t.numel() * t.element_size()
            v = slab[offs[n]:offs[n] + nb].view(t.dtype)
            v.copy_(t)
            setattr(self, n, v)
            del t
        self._slab = slab
        torch.cuda.empty_cache()


engine.ProgressState = SlabState


def main():
    args = bench.parse([])
    args.workload = "config2_n5"
    d = bench.Dist()
    for name in os.environ.get("WLS", "progress_send").split(","):
        r = bench.run_workload(name, args, d, 20, 5)
        print(f"slab {int(SLAB)} skew {SKEW:6d} {name:20s} kernel {r['kernel_ms']:.4f} ms  "
              f"frac {r['hbm_frac']:.3f}  checksum {r['checksum']}", flush=True)


if __name__ == "__main__":
    main()
