#!/usr/bin/env python3
"""DESIGN.md §6's measurement table from one bench log and the committed PMC:

  python scripts/design_table.py profiles/r05/bench_fin.log [profiles/r05_pmc.json]

Per workload: value, the bench's HIP-event kernel time, the fraction of the
bound with the algorithmic bytes per unit, the PMC traffic per launch (2 x
FETCH_SIZE + WRITE_SIZE, as calibrated) over the algorithmic bytes, vector-
memory instructions per 64-group tile, SQ_WAIT_ANY / SQ_WAVE_CYCLES and the
waves/SIMD of the code objects (the bench line's occupancy entry)."""
import json
import sys

ROWS = [
    ("config2_n5", "**config 2, 5 voters (headline)**"),
    ("config2_n7", "config 2, 7 voters"),
    ("config3_joint_packed", "config 3 joint, through the packer"),
    ("config3_joint", "config 3 joint, generator-bucketed"),
    ("config3_joint_rot", "config 3 joint, rotated slots"),
    ("config4_repl", "config 4 replication round"),
    ("config4_repl_joint", "config 4, joint 6 slots"),
    ("config5_elec", "config 5 election"),
    ("config5_prevote_cq", "config 5 + PreVote + CheckQuorum"),
    ("progress_step", "**Progress step** (16M × 5)"),
    ("progress_step_n7", "Progress step, S = 7"),
    ("progress_step_joint", "Progress step, joint 5+5 over 6"),
    ("progress_send", "Progress send"),
    ("propose", "propose (ABI 6)"),
    ("heartbeat", "heartbeat (ABI 6)"),
    ("switch_config", "switchToConfig (ABI 7)"),
    ("check_quorum", "CheckQuorum"),
    ("confchange", "confchange"),
    ("ready_collect", "ready_collect (3 kernels)"),
]


def main():
    line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
    d = json.loads(line)
    pmc = json.load(open(sys.argv[2] if len(sys.argv) > 2 else "profiles/r05_pmc.json"))
    traffic = json.load(open("profiles/pmc_traffic.json"))
    aux = dict(d["aux"])
    aux["config2_n5"] = {"value": d["value"], "kernel_ms": d["roofline"]["kernel_ms"],
                         "hbm_frac": d["roofline"]["frac"],
                         "bytes_per_unit": d["roofline"]["bytes_per_unit"],
                         "occupancy": {k: v for k, v in json.load(open(
                             "profiles/kernel_resources.json")).items()
                             if k.startswith("void qe::k_cv_stream<5, 0,")}}
    print("| workload | value | kernel (bench HIP events) | frac of bound (algorithmic B/unit) "
          "| PMC traffic / launch (× algorithmic) | vmem/tile | wait | waves/SIMD |")
    print("|---|---|---|---|---|---|---|---|")
    for wl, label in ROWS:
        a = aux.get(wl)
        if a is None:
            continue
        v = a.get("roofline_valu") or {}
        if "cycles_frac" in v:
            frac = (f"VALU: **{v['cycles_frac']:.2f}** of SIMD cycles "
                    f"({v['insts_frac_measured_clock']:.2f} by count)")
        else:
            frac = f"{a['hbm_frac']:.3f} ({a['bytes_per_unit']:.0f})"
        t = traffic.get(wl, {})
        tr = (f"{t['hbm_bytes_per_launch'] / 1e9:.2f} GB ({t['traffic_over_algorithmic']:.2f})"
              if "traffic_over_algorithmic" in t else "—")
        # the PMC record the workload's traffic entry names (its latest profile)
        prof = t.get("profile")
        p = (json.load(open(prof)) if prof else {}).get(wl) or pmc.get(wl, {})
        # per 64-unit tile: units per launch = algorithmic bytes / bytes per unit
        units = (t["algorithmic_bytes_per_launch"] / a["bytes_per_unit"]
                 if "algorithmic_bytes_per_launch" in t and a.get("bytes_per_unit") else None)
        vm = ((p["SQ_INSTS_VMEM_RD"] + p["SQ_INSTS_VMEM_WR"]) / (units / 64)
              if units and "SQ_INSTS_VMEM_RD" in p else None)
        wait = p["SQ_WAIT_ANY"] / p["SQ_WAVE_CYCLES"] if p.get("SQ_WAVE_CYCLES") else None
        occ = a.get("occupancy") or {}
        wps = ", ".join(str(o["waves_per_simd"]) for o in occ.values()) or "—"
        print(f"| {label} | {a['value']:.3g} | {a['kernel_ms']:.3f} ms | {frac} | {tr} | "
              f"{'—' if vm is None else f'{vm:.0f}'} | {'—' if wait is None else f'{wait:.2f}'} | {wps} |")


if __name__ == "__main__":
    main()
