#!/usr/bin/env python3
"""Does a workload's kernel time depend on what ran before it in the process?
(round 6: progress_send / switch_config time 1.26 / 1.69 ms as bench.py's
headline workload, 1.10 / 1.38 ms as aux workloads after the others.)

  ORDER=progress_send,progress_send,config2_n5,progress_send python scripts/order_probe.py

Runs bench.run_workload for each name in ORDER in one process and prints
the HIP-event kernel time of each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from etcd_amd import engine  # noqa: E402

bench.engine = engine


def main():
    args = bench.parse([])
    args.workload = "config2_n5"
    d = bench.Dist()
    import torch
    for name in os.environ.get("ORDER", "progress_send,progress_send").split(","):
        if name.startswith("alloc"):  # allocN: N GiB allocated, written, freed
            t = torch.empty(int(name[5:]) << 30, dtype=torch.uint8, device=d.dev)
            t.fill_(1)
            torch.cuda.synchronize(d.dev)
            del t
            torch.cuda.empty_cache()
            print(name, flush=True)
            continue
        if name.startswith("hold"):  # holdN: N GiB allocated and kept
            globals().setdefault("_held", []).append(
                torch.empty(int(name[4:]) << 30, dtype=torch.uint8, device=d.dev))
            print(name, flush=True)
            continue
        r = bench.run_workload(name, args, d, 20, 5)
        print(f"{name:20s} kernel {r['kernel_ms']:.4f} ms  frac {r['hbm_frac']:.3f}", flush=True)


if __name__ == "__main__":
    main()
