#!/usr/bin/env python3
"""Register / LDS / scratch budget and occupancy of the built kernels, from
the code objects inside the in-tree objects (etcd_amd/build/*.o: the
.hip_fatbin section, unbundled for gfx950, its AMDGPU metadata note).

  python scripts/kernel_resources.py [pattern ...]  -> profiles/kernel_resources.json
  QE_KR_OUT=profiles/x.json python scripts/kernel_resources.py PATTERN  -> another file

Waves per SIMD (gfx950, wave64): min(8, 512 // vgpr_alloc) with VGPRs+AGPRs
allocated in granules of 8, and the LDS bound: floor(160 KiB / LDS per
block) blocks per CU x waves per block / 4 SIMDs.  bench.py reads the entry
of each workload's dominant kernel into its aux line (waves_per_simd).
"""
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
LDS_PER_CU = 160 * 1024


def code_object(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fat")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True, stderr=subprocess.DEVNULL)
    return co


def kernels(co):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out = {}
    for blk in notes.split("  - .agpr_count:")[1:]:
        g = lambda k: re.search(r"\." + k + r":\s+(\S+)", blk)  # noqa: E731
        name = g("name")
        if not name:
            continue
        agpr = int(blk.split("\n", 1)[0].strip())
        vgpr = int(g("vgpr_count").group(1))
        lds = int(g("group_segment_fixed_size").group(1))
        wg = int(g("max_flat_workgroup_size").group(1))
        alloc = -(-(vgpr + agpr) // 8) * 8
        w_vgpr = min(8, 512 // max(alloc, 1))
        wpb = max(1, wg // 64)
        w_lds = (LDS_PER_CU // lds) * wpb / 4 if lds else 8
        out[name.group(1)] = {
            "vgpr": vgpr, "agpr": agpr, "sgpr": int(g("sgpr_count").group(1)),
            "vgpr_spill": int(g("vgpr_spill_count").group(1)),
            "sgpr_spill": int(g("sgpr_spill_count").group(1)),
            "scratch_bytes": int(g("private_segment_fixed_size").group(1)),
            "lds_bytes": lds, "max_wg": wg,
            "waves_per_simd": min(w_vgpr, w_lds), "waves_per_simd_vgpr": w_vgpr,
            "waves_per_simd_lds": w_lds,
        }
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                       text=True, check=True)
    return r.stdout.split("\n")


def main():
    # default: the instantiations the bench workloads launch
    pats = sys.argv[1:] or ["qe::k_progress_step<5, unsigned char, false, false, 4, false,",
                            "qe::k_progress_step<7, unsigned char, false, false, 4, false,",
                            "qe::k_progress_step<6, unsigned char, true, true, 4, false,",
                            "qe::k_progress_send<5,", "qe::k_check_quorum<5,",
                            "qe::k_propose<5, unsigned char, false, false, false,",
                            "qe::k_switch_config<5, unsigned char, true, false, false,",
                            "qe::k_heartbeat<5,",
                            "qe::k_cv_stream<5, 0,", "qe::k_cv_stream<7, 0,", "qe::k_cv_stream<10, 2,",
                            "qe::k_repl_stream<5,", "qe::k_repl_stream<6,", "qe::k_confchange<5>",
                            "qe::k_collect", "qe::k_election<5,"]
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for obj in sorted(glob.glob(os.path.join(ROOT, "etcd_amd", os.environ.get("QE_KR_BUILD", "build"), "*.o"))):
            try:
                co = code_object(obj, tmp)
            except subprocess.CalledProcessError:
                continue  # host-only object
            ks = kernels(co)
            for mangled, dem in zip(ks, demangle(list(ks))):
                if any(p in dem for p in pats):
                    res[dem] = dict(ks[mangled], object=os.path.basename(obj))
    path = os.path.join(ROOT, os.environ.get("QE_KR_OUT", "profiles/kernel_resources.json"))
    with open(path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(f"{len(res)} kernels -> {path}")


if __name__ == "__main__":
    main()
