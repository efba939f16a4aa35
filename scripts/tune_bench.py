#!/usr/bin/env python3
"""Interleaved in-process A/B of launch knobs over bench.py workloads.

  TUNE_WL=config4_repl,progress_step TUNE_TPW=-1,1,2,4 TUNE_NT=0,3 python scripts/tune_bench.py

For each workload: set up once (bench.setup), then ROUNDS x (each knob
variant x LAUNCHES timed launches with HIP events on the launch stream).
Prints one line per (workload, variant): median / min ms and GB/s
(algorithmic bytes)."""
import itertools
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from etcd_amd import engine  # noqa: E402

bench.engine = engine  # bench.py imports the engine lazily in its main()

ROUNDS, LAUNCHES = 5, 15


def main():
    d = bench.Dist()
    wls = os.environ.get("TUNE_WL", "config4_repl").split(",")
    tpws = [int(x) for x in os.environ.get("TUNE_TPW", "-1,1,2,4,8").split(",")]
    nts = [int(x) for x in os.environ.get("TUNE_NT", "3").split(",")]
    # TUNE_KNOB=name=v1,v2 (e.g. repl_kernel=0,1): one more qe_tune axis
    kname, kvals = "", [None]
    if os.environ.get("TUNE_KNOB"):
        kname, kv = os.environ["TUNE_KNOB"].split("=")
        kvals = [int(x) for x in kv.split(",")]
    for wl in wls:
        desc, G, S, kind = bench.WORKLOADS[wl]
        stats = engine.stats_buffer(d.dev)
        step, bpu, units, _, keep = bench.setup(wl, G, S, kind, d, stats)
        prep = keep.get("prepare") or (lambda: None)  # per-launch state restore
        variants = list(itertools.product(tpws, nts, kvals))
        res = {v: [] for v in variants}
        for _ in range(ROUNDS):
            for v in variants:
                engine.tune("tiles_per_wave", v[0])
                engine.tune("nontemporal", v[1])
                if kname:
                    engine.tune(kname, v[2])
                for _ in range(3):
                    prep()
                    step()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(LAUNCHES)]
                for a, b in ev:
                    prep()
                    a.record()
                    step()
                    b.record()
                torch.cuda.synchronize()
                res[v] += [a.elapsed_time(b) for a, b in ev]
        engine.tune("tiles_per_wave", -1)
        engine.tune("nontemporal", 3)
        if kname:
            engine.tune(kname, -1)
        for v in variants:
            ms = np.array(res[v])
            kx = f" {kname}={v[2]}" if kname else ""
            print(f"{os.path.basename(engine._lib.LIB_PATH)} {wl} tpw={v[0]} nt={v[1]}{kx} median {np.median(ms):.4f} ms  min {ms.min():.4f}  "
                  f"{bpu * units / np.median(ms) / 1e6:.0f} GB/s", flush=True)
        del keep
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
