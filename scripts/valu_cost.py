#!/usr/bin/env python3
"""Cycle-weighted VALU bound of the election kernels.

SQ_INSTS_VALU counts wave64 VALU instructions; on gfx950 neither
SQ_ACTIVE_INST_VALU nor SQ_THREAD_CYCLES_VALU weights them by issue cost:
scripts/valu_probe.hip runs 32 independent instructions of one kind per
iteration at 8 waves/SIMD, and for every kind both counters equal the
instruction count (x64 for THREAD_CYCLES), while the time doubles for
v_mul_lo_u32, v_mul_u32_u24 and v_bcnt_u32_b32.  So the cost of each kind is
measured instead, as shader cycles per wave64 instruction per SIMD:

    cost(kind) = (GRBM_GUI_ACTIVE / 8 XCDs) / (SQ_INSTS_VALU / 1024 SIMDs)

from the probe's own --pmc pass, and the election's VALU time is its
instruction count weighted by the mix of its per-step loop (the static loop
body of the code object whose VALU count matches the measured dynamic count
per wave-step; opcodes the probe did not cover take the v_add_u32 cost and
are listed).  Reported per workload:

    insts_frac  = insts/SIMD x cost(v_add_u32) / kernel cycles  (the r04 figure,
                  now at the measured full-rate cost and shader clock)
    cycles_frac = insts/SIMD x mix-weighted cost / kernel cycles

usage: valu_cost.py <probe dir (valu_pmc/)> [workload dir (valu_config5_elec/,
       valu_config5_prevote_cq/); default the probe dir]
       -> profiles/valu_cost.json (bench.py adds cycles_frac to roofline_valu)
"""
import collections
import csv
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import kernel_resources as kr  # noqa: E402

XCDS, SIMDS = 8, 1024
PROBE_KINDS = {  # k_valu<KIND, T> -> opcode prefix it issues
    0: "v_add_u32", 1: "v_xor_b32", 2: "v_mul_lo_u32", 3: "v_mul_u32_u24",
    4: "v_bcnt_u32_b32", 5: "v_bitop3_b32", 6: "v_cndmask_b32", 7: "v_mul_lo_u16",
    8: "v_add3_u32", 9: "v_mad_u64_u32", 10: "v_lshl_add_u64", 11: "v_lshrrev_b64",
    12: "v_mov_b32", 13: "v_cmp_gt_u32", 14: "v_and_b32", 15: "v_or3_b32", 16: "v_lshrrev_b32",
    17: "v_sub_u32", 18: "v_cndmask_b32_e32", 19: "v_readlane_b32", 20: "v_writelane_b32",
    21: "v_min_u32", 22: "v_max_u32", 23: "v_lshlrev_b32", 24: "v_alignbit_b32",
    25: "v_and_or_b32"}
# opcodes priced as a probed one of the same form: every 32-bit compare
# writes a lane mask as v_cmp_gt_u32 does
ALIASES = (("v_cmp_", "v_cmp_gt_u32"),)
WORKLOADS = {  # workload -> (object, kernel symbol, wave-steps per launch)
    "config5_elec": ("qe_inst_5.o", "_ZN2qe10k_electionILi5EhLi0EEEvNS_5EArgsE", (2 << 20) // 64 * 64),
    "config5_prevote_cq": ("qe_inst_5.o", "_ZN2qe10k_electionILi5EhLi3EEEvNS_5EArgsE",
                           (2 << 20) // 64 * 64),
}


def pmc(path):
    """Per kernel name: counter -> mean value per dispatch."""
    rows = list(csv.DictReader(open(path)))
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        tot[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in tot.items()}


def probe_costs(d):
    out = {}
    for name, c in pmc(os.path.join(d, "valu_pmc", "v_counter_collection.csv")).items():
        m = re.match(r"void k_valu<(\d+)", name)
        if m and c.get("SQ_INSTS_VALU"):
            cyc = c["GRBM_GUI_ACTIVE"] / XCDS
            out[PROBE_KINDS[int(m.group(1))]] = {
                "cycles_per_inst": cyc / (c["SQ_INSTS_VALU"] / SIMDS),
                "active_inst_over_insts": c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"],
                "thread_cycles_over_insts": c["SQ_THREAD_CYCLES_VALU"] / c["SQ_INSTS_VALU"]}
    return out


def step_loop_mix(obj, sym, dyn_per_step):
    co = kr.code_object(os.path.join(ROOT, "etcd_amd", "build", obj), tempfile.mkdtemp())
    d = subprocess.run([f"{kr.LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                        "--symbolize-operands", co], check=True, capture_output=True,
                       text=True).stdout
    i = d.index("<" + sym + ">:")
    m = re.compile(r"^[0-9a-f]+ <_Z", re.M).search(d, i + 10)
    ins = [ln.split("//")[0].strip() for ln in d[i:m.start() if m else len(d)].split("\n")[1:]]
    ins = [ln for ln in ins if ln]
    lab = {}
    for k, ln in enumerate(ins):
        mm = re.match(r"(?:[0-9a-f]+ )?<(L\d+)>:", ln)
        if mm:
            lab[mm.group(1)] = k
    loops = []
    for k, ln in enumerate(ins):
        mm = re.match(r"(s_cbranch_\w+|s_branch)\s+<?(L\d+)>?", ln)
        if mm and mm.group(2) in lab and lab[mm.group(2)] < k:
            a = lab[mm.group(2)]
            ops = [x.split()[0] for x in ins[a:k + 1] if x.startswith("v_")]
            loops.append((abs(len(ops) - dyn_per_step), a, k, ops))
    _, a, b, ops = min(loops)
    return collections.Counter(ops), (a, b)


def base(op):
    """Encodings fold into the opcode (e64 = VOP3 of the same operation).
    The probe's v_cndmask_b32_e32 chain (implicit VCC) measured ~24 cycles
    per instruction, an outlier we do not understand (compiled code issues
    that form everywhere); it is recorded in the probe table but the e64 cost
    prices every v_cndmask_b32."""
    op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    return op


def cost_of(b, costs):
    if b in costs:
        return costs[b]["cycles_per_inst"]
    for prefix, probed in ALIASES:
        if b.startswith(prefix) and probed in costs and b[-4:] in ("_u32", "_i32"):
            return costs[probed]["cycles_per_inst"]
    return None


def main():
    d = sys.argv[1]
    dw = sys.argv[2] if len(sys.argv) > 2 else d
    costs = probe_costs(d)
    full = costs["v_add_u32"]["cycles_per_inst"]
    out = {"probe": costs, "source": os.path.relpath(d, ROOT),
           "workload_source": os.path.relpath(dw, ROOT), "workloads": {}}
    for wl, (obj, sym, wave_steps) in WORKLOADS.items():
        f = os.path.join(dw, f"valu_{wl}", "v_counter_collection.csv")
        if not os.path.exists(f):
            continue
        ks = {k: v for k, v in pmc(f).items() if "k_election" in k}
        (kname, c), = ks.items()
        insts = c["SQ_INSTS_VALU"]
        cycles = c["GRBM_GUI_ACTIVE"] / XCDS
        dyn = insts / wave_steps
        mix, region = step_loop_mix(obj, sym, dyn)
        n = sum(mix.values())
        w, assumed = 0.0, {}
        for op, k in mix.items():
            b = base(op)
            hit = cost_of(b, costs)
            if hit is None:
                assumed[b] = assumed.get(b, 0) + k / n
                hit = full
            w += k / n * hit
        per_simd = insts / SIMDS
        out["workloads"][wl] = {
            "kernel": kname, "valu_insts_per_launch": insts, "kernel_cycles": cycles,
            "valu_per_wave_step": dyn, "step_loop_valu": n, "step_loop_region": region,
            "mix_top": {base(k): v / n for k, v in mix.most_common(12)},
            "avg_cycles_per_inst": w, "full_rate_cycles": full,
            "insts_frac": per_simd * full / cycles, "cycles_frac": per_simd * w / cycles,
            "assumed_full_rate_share": sum(assumed.values()), "assumed_ops": sorted(assumed)}
    path = os.path.join(ROOT, "profiles", "valu_cost.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for wl, r in out["workloads"].items():
        print(f"{wl:20s} VALU/wave-step {r['valu_per_wave_step']:.1f} (loop {r['step_loop_valu']})"
              f"  avg {r['avg_cycles_per_inst']:.3f} cyc (full {full:.3f})"
              f"  insts_frac {r['insts_frac']:.3f}  cycles_frac {r['cycles_frac']:.3f}"
              f"  assumed {r['assumed_full_rate_share']:.2f}")
    print("->", path)


if __name__ == "__main__":
    main()
