#!/usr/bin/env python3
"""Fold a gpurun rocprofv3 run (gpurun_out/prof/{kt,fetch,write}) into the
committed evidence under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_summary.json   per-kernel FETCH_SIZE / WRITE_SIZE means
  profiles/pmc_traffic.json         HBM bytes per launch of each bench
                                    workload's dominant kernel (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream,
so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  The doubling was
calibrated on this kernel's own access pattern: 2 * FETCH_SIZE equals the
algorithmic read bytes of qe_commit_vote within 0.01 %.

usage: python scripts/summarize_profile.py <tag> [prof_dir]
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench workload -> kernel-name prefix of its dominant kernel
DOMINANT = {
    "config2_n5": "void qe::k_cv_stream<5, 0,",
    "config2_n7": "void qe::k_cv_stream<7, 0,",
    "config3_joint": "void qe::k_cv_stream<10, 2,",  # bucketed + rotated runs share it
    "config4_repl": "void qe::k_repl_stream<5,",
    "config5_elec": "void qe::k_election<5,",
    "progress_step": "void qe::k_progress_step<5,",
    "confchange": "void qe::k_confchange<",
}


def counters(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        agg.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    tag = sys.argv[1]
    prof = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(prof, "kt", "kt_kernel_stats.csv"),
                os.path.join(out, f"{tag}_kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(prof, "kt", "kt_kernel_stats.csv")))}
    fetch = counters(os.path.join(prof, "fetch", "fetch_counter_collection.csv"))
    write = counters(os.path.join(prof, "write", "write_counter_collection.csv"))
    summary = {}
    for k in sorted(set(fetch) | set(write)):
        if "qe::" not in k:
            continue
        summary[k] = {"FETCH_SIZE_KiB": fetch.get(k), "WRITE_SIZE_KiB": write.get(k),
                      "avg_ns": float(stats[k]["AverageNs"]) if k in stats else None,
                      "calls": int(stats[k]["Calls"]) if k in stats else None}
    with open(os.path.join(out, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    traffic = {}
    for wl, prefix in DOMINANT.items():
        for k, v in summary.items():
            if k.startswith(prefix) and v["FETCH_SIZE_KiB"] is not None and v["WRITE_SIZE_KiB"] is not None:
                traffic[wl] = {
                    "kernel": k, "profile": f"profiles/{tag}_pmc_summary.json",
                    "hbm_bytes_per_launch": (2 * v["FETCH_SIZE_KiB"] + v["WRITE_SIZE_KiB"]) * 1024,
                    "rocprof_avg_ns": v["avg_ns"],
                }
    with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    for wl, t in traffic.items():
        print(wl, f"{t['hbm_bytes_per_launch'] / 1e9:.3f} GB/launch", t["rocprof_avg_ns"], "ns")


if __name__ == "__main__":
    main()
