#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration factors by access width (scripts/
pmc_calib.hip): factor = known bytes / (counter KiB x 1024), per kernel,
median over its launches.  usage: pmc_calib.py <probe stdout> <fetch dir> <write dir> <out.json>"""
import csv
import glob
import json
import sys

KMAP = {"rd<unsigned char>": "r1", "rd<unsigned short>": "r2", "rd<unsigned int>": "r4",
        "rd<unsigned long long>": "r8", "r16": "r16", "r8h": "r8h", "r16ring": "r16ring",
        "wr<unsigned char>": "w1", "wr<unsigned int>": "w4", "wr<unsigned long long>": "w8",
        "w16": "w16", "w4ring": "w4ring", "w16ring": "w16ring"}


def short(kname):
    k = kname.split("(")[0].replace("void ", "").strip()
    return KMAP.get(k, k)


def counters(d):
    acc = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc.setdefault((short(r["Kernel_Name"]), r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in acc.items()}


def main():
    known = {}
    for line in open(sys.argv[1]):
        p = line.split()
        if len(p) == 3 and p[1] == "known_bytes":
            known[p[0]] = float(p[2])
    c = counters(sys.argv[2])
    c.update(counters(sys.argv[3]))
    out = {}
    for name, b in known.items():
        cn = "FETCH_SIZE" if name.startswith("r") else "WRITE_SIZE"
        v = c.get((name, cn))
        if v:
            out[name] = {"counter": cn, "known_bytes": b, "counter_bytes": v * 1024,
                         "factor": b / (v * 1024)}
            print(f"{name:8s} {cn} x{b / (v * 1024):.3f}  (known {b / 1e6:.1f} MB, counted {v * 1024 / 1e6:.1f} MB)")
    json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
