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
Calibrated on this box's own access widths (scripts/pmc_calib.hip,
profiles/r04/pmc_calib.json): FETCH_SIZE reports exactly half of the bytes
a read moves from memory for every row width the engine uses (1, 2, 4, 8
and 16 B per lane: x2.000).  A row read at half density (every other u64,
or 16 B of each lane's 32-B ring) still moves every sector it touches:
FETCH_SIZE then equals the bytes the lanes asked for, which is half of the
sectors moved -- x2 again for the memory-side bytes.  So every kernel's
read traffic is 2 x FETCH_SIZE.  WRITE_SIZE counts whole 32-B sectors: exact for full rows
(x1.000 for 4-, 8-, 16-B lanes), 32 B for a 4-B append into a lane's
32-B ring (x0.125) and for 16 B of it (x0.5) -- it is the memory-side
write traffic as is.  (Rounds 1-3 used x1 for the narrow-access kernels,
which undercounted their reads by half; check_quorum's figure fell below
its algorithmic bytes.)  usage: summarize_workloads.py <tag> [dir] [bench.log ...]:
with a bench JSON line, every workload's traffic is checked against its
algorithmic bytes (units x bytes_per_unit) and a figure below it is refused.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# workload -> (kernel-name prefix of the dominant kernel, FETCH_SIZE factor:
# 2 for every kernel, profiles/r04/pmc_calib.json)
DOMINANT = {
    "config2_n5": ("void qe::k_cv_stream<5, 0,", 2),
    "config2_n7": ("void qe::k_cv_stream<7, 0,", 2),
    "config3_joint": ("void qe::k_cv_stream<10, 2,", 2),
    "config3_joint_rot": ("void qe::k_cv_stream<10, 2,", 2),
    "config3_joint_packed": ("void qe::k_cv_stream<10, 2,", 2),
    # check_quorum: dword rows of the peer words (256 B per row instruction)
    # and byte rows: 64-B requests, FETCH_SIZE x 1
    "check_quorum": ("void qe::k_check_quorum<5,", 2),
    "config4_repl": ("void qe::k_repl_stream<5,", 2),
    "config5_elec": ("void qe::k_election<5, unsigned char, 0>", 2),
    "config5_prevote_cq": ("void qe::k_election<5, unsigned char, 3>", 2),
    "progress_step": ("void qe::k_progress_step<5, unsigned char, false, false, 4, false,", 2),
    # confchange: its ID block and u64 rows are read 512 B per instruction
    # (128-B requests): 2 x FETCH_SIZE = 75.0 B/group = its algorithmic reads
    # (r02h); round-2 summaries before r02h used 1
    "confchange": ("void qe::k_confchange<5>", 2),
    "config4_repl_joint": ("void qe::k_repl_stream<6, true, true,", 2),
    # ready_collect: all three kernels of one qe_collect (count, scan, scatter)
    "ready_collect": (("void qe::k_collect_count", "void qe::k_collect_scan",
                       "void qe::k_collect_scatter"), 2),
    "progress_send": ("void qe::k_progress_send<5,", 2),
    # (round 6: a trailing template flag selects the 16-bit Inflights form)
    "propose": ("void qe::k_propose<5, unsigned char, false, false, false,", 2),
    # the default one-tile-per-wave kernel (round 6's pipelined k_heartbeat_pipe
    # measured slower, profiles/r06/heartbeat_ab.txt)
    "heartbeat": ("void qe::k_heartbeat<5, unsigned char>", 2),
    "switch_config": ("void qe::k_switch_config<5, unsigned char, true, false, false,", 2),
    "progress_step_n7": ("void qe::k_progress_step<7, unsigned char, false, false, 4, false,", 2),
    "progress_step_joint": ("void qe::k_progress_step<6, unsigned char, true, true, 4, false,", 2),
}


def counters(path):
    agg = {}
    for f in glob.glob(path, recursive=True):
        for r in csv.DictReader(open(f)):
            agg.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def algorithmic_bytes(bench_log):
    """workload -> algorithmic bytes per launch from a bench.py JSON line
    (the headline and every aux workload: bytes_per_unit x units)."""
    line = [l for l in open(bench_log) if l.startswith("{")][-1]
    d = json.loads(line)
    out = {}
    wl = d["config"]["workload"].split(":")[0]
    r = d["roofline"]
    out[wl] = r["achieved"] * 1e9 * r["kernel_ms"] / 1e3
    for k, v in d.get("aux", {}).items():
        if "achieved_GBs" in v and "kernel_ms" in v:
            out[k] = v["achieved_GBs"] * 1e9 * v["kernel_ms"] / 1e3
    return out


def main():
    tag = sys.argv[1]
    base = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "profw")
    algo = {}
    for log in sys.argv[3:]:  # one or more bench logs
        algo.update(algorithmic_bytes(log))
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
        for p in ("fetch", "write", "sq", "vmem", "stall"):
            c.update(counters(os.path.join(d, p, "**", "*counter_collection.csv")))
        prefixes = prefix if isinstance(prefix, tuple) else (prefix,)
        bare = lambda x: x[5:] if x.startswith("void ") else x  # noqa: E731
        names = [next((k for k in stats if bare(k).startswith(bare(p_))), None) for p_ in prefixes]
        if not all(names):
            continue
        k = " + ".join(names)
        row = {"kernel": k, "avg_ns": sum(float(stats[n]["AverageNs"]) for n in names),
               "calls": int(stats[names[-1]]["Calls"])}
        for (kn, cn), v in c.items():  # a multi-kernel workload: the sum per launch
            if kn in names:
                row[cn] = row.get(cn, 0.0) + v
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
            if wl in algo:
                t["algorithmic_bytes_per_launch"] = algo[wl]
                t["traffic_over_algorithmic"] = t["hbm_bytes_per_launch"] / algo[wl]
                if t["hbm_bytes_per_launch"] < 0.995 * algo[wl]:
                    raise SystemExit(f"{wl}: PMC traffic {t['hbm_bytes_per_launch'] / 1e9:.3f} GB "
                                     f"is below its algorithmic {algo[wl] / 1e9:.3f} GB -- "
                                     f"a wrong counter correction, refused")
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
    # where the dominant kernel's wave cycles go (the stall pass), each over SQ_WAVE_CYCLES
    for wl, row in summary.items():
        if "SQ_WAIT_INST_ANY" in row and row.get("SQ_WAVE_CYCLES"):
            wc = row["SQ_WAVE_CYCLES"]
            print(f"{wl:20s} " + "  ".join(
                f"{k[3:]} {row[k] / wc:.3f}" for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                        "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                                                        "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS") if k in row))


if __name__ == "__main__":
    main()
