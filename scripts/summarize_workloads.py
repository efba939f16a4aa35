#!/usr/bin/env python3
"""Fold scripts/gpu_profile_workloads.sh output (gpurun_out/profw/<wl>/...)
into the committed evidence:

  profiles/<tag>/<wl>_kernel_stats.csv   rocprofv3 --kernel-trace --stats
  profiles/<tag>_pmc.json                per workload: the dominant kernel's
                                         average duration, FETCH_SIZE,
                                         WRITE_SIZE and SQ counters per launch
  profiles/pmc_traffic.json              what bench.py reads: HBM bytes and
                                         VALU instructions per launch

HBM bytes (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are KiB.
FETCH_SIZE counts each memory-side read request as 64 B; gfx950's wide
coalesced streams issue 128-B requests, so for the streaming kernels
(k_cv_stream, k_repl_stream) the read bytes are 2 x FETCH_SIZE, calibrated
in round 1 (2 x FETCH_SIZE = algorithmic reads within 0.01 %).  Kernels
whose reads are mostly narrow or scattered (Progress step: 8-B Inflights
rows, byte loads; election) issue 64-B requests and read
FETCH_SIZE x 1 (checked for the Progress step against its access
inventory).  usage: summarize_workloads.py <tag> [dir]
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# workload -> (kernel-name prefix of the dominant kernel, FETCH_SIZE factor)
DOMINANT = {
    "config2_n5": ("void qe::k_cv_stream<5, 0,", 2),
    "config2_n7": ("void qe::k_cv_stream<7, 0,", 2),
    "config3_joint": ("void qe::k_cv_stream<10, 2,", 2),
    "config3_joint_rot": ("void qe::k_cv_stream<10, 2,", 2),
    "config3_joint_packed": ("void qe::k_cv_stream<10, 2,", 2),
    # check_quorum: dword rows of the peer words (256 B per row instruction)
    # and byte rows: 64-B requests, FETCH_SIZE x 1
    "check_quorum": ("void qe::k_check_quorum<5,", 1),
    "config4_repl": ("void qe::k_repl_stream<5,", 2),
    "config5_elec": ("void qe::k_election<5, unsigned char, 0>", 1),
    "config5_prevote_cq": ("void qe::k_election<5, unsigned char, 3>", 1),
    "progress_step": ("void qe::k_progress_step<5, unsigned char, false, false, 4, false,", 1),
    # confchange: its ID block and u64 rows are read 512 B per instruction
    # (128-B requests): 2 x FETCH_SIZE = 75.0 B/group = its algorithmic reads
    # (r02h); round-2 summaries before r02h used 1
    "confchange": ("void qe::k_confchange<5>", 2),
    "config4_repl_joint": ("void qe::k_repl_stream<6, true, true,", 2),
    "ready_collect": ("qe::k_collect_scatter", 1),
    "progress_send": ("void qe::k_progress_send<5,", 1),
}


def counters(path):
    agg = {}
    for f in glob.glob(path, recursive=True):
        for r in csv.DictReader(open(f)):
            agg.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    tag = sys.argv[1]
    base = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "profw")
    outd = os.path.join(ROOT, "profiles", tag)
    os.makedirs(outd, exist_ok=True)
    summary, traffic = {}, {}
    for wl, (prefix, ffac) in DOMINANT.items():
        d = os.path.join(base, wl)
        kts = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
        if not kts:
            continue
        shutil.copy(kts[0], os.path.join(outd, f"{wl}_kernel_stats.csv"))
        stats = {r["Name"]: r for r in csv.DictReader(open(kts[0]))}
        c = {}
        for p in ("fetch", "write", "sq", "vmem"):
            c.update(counters(os.path.join(d, p, "**", "*counter_collection.csv")))
        names = [k for k in stats if k.startswith(prefix)]
        if not names:
            continue
        k = names[0]
        row = {"kernel": k, "avg_ns": float(stats[k]["AverageNs"]), "calls": int(stats[k]["Calls"])}
        for (kn, cn), v in c.items():
            if kn == k:
                row[cn] = v
        summary[wl] = row
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            t = {"kernel": k, "profile": f"profiles/{tag}_pmc.json",
                 "fetch_factor": ffac,
                 "hbm_bytes_per_launch": (ffac * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024,
                 "rocprof_avg_ns": row["avg_ns"]}
            if "SQ_INSTS_VALU" in row:
                t["valu_insts_per_launch"] = row["SQ_INSTS_VALU"]
                t["salu_insts_per_launch"] = row.get("SQ_INSTS_SALU")
                t["waves_per_launch"] = row.get("SQ_WAVES")
            if "SQ_INSTS_VMEM_RD" in row:
                t["vmem_rd_per_launch"] = row["SQ_INSTS_VMEM_RD"]
                t["vmem_wr_per_launch"] = row.get("SQ_INSTS_VMEM_WR")
            traffic[wl] = t
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # merge: a run that profiled some workloads replaces only their entries
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    merged = json.load(open(tp)) if os.path.exists(tp) else {}
    merged.update(traffic)
    with open(tp, "w") as f:
        json.dump(merged, f, indent=1)
    for wl, t in traffic.items():
        print(f"{wl:20s} {t['hbm_bytes_per_launch'] / 1e9:8.3f} GB/launch  {t['rocprof_avg_ns'] / 1e6:.4f} ms"
              f"  VALU {t.get('valu_insts_per_launch', 0):.3e}")


if __name__ == "__main__":
    main()
