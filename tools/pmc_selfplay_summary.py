#!/usr/bin/env python3
"""Summarise tools/pmc_selfplay.sh for the config-3 self-play kernels into one JSON
(profiles/). Per kernel: average duration (kernel trace), HBM bytes per launch
(FETCH_SIZE KB x1024 x2 gfx950 correction + WRITE_SIZE KB x1024, MI355X_MICROARCH.md HBM
section), SQ instruction counts per wave and the fraction of wave time spent waiting on
memory/LDS counters (SQ_WAIT_ANY / SQ_WAVE_CYCLES)."""
import csv
import glob
import json
import os
import re
import sys

KERNELS = ("k_select", "k_leaf_mask", "k_nn_forward", "k_backup", "k_commit")


def per_kernel(d):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"k_\w+", r.get("Kernel_Name", ""))
            if not m or m.group(0) not in KERNELS:
                continue
            k, disp = m.group(0), int(r["Dispatch_Id"])
            acc.setdefault(k, {}).setdefault(disp, {})
            c = r["Counter_Name"]
            acc[k][disp][c] = acc[k][disp].get(c, 0.0) + float(r["Counter_Value"])
    out = {}
    for k, disps in acc.items():
        names = {c for v in disps.values() for c in v}
        out[k] = {c: sum(v.get(c, 0.0) for v in disps.values()) / len(disps) for c in names}
    return out


def durations(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"k_\w+", r["Name"])
            if m and m.group(0) in KERNELS:
                out[m.group(0)] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def main():
    root, rnd = sys.argv[1], sys.argv[2]
    fe, wr, sq, du = (per_kernel(os.path.join(root, "fetch")), per_kernel(os.path.join(root, "write")),
                      per_kernel(os.path.join(root, "sq")), durations(os.path.join(root, "trace")))
    res = {"round": rnd, "workload": "config 3: 32768 self-play games, numMCTSSims=100 (genbu args), "
           "one select/network/backup/commit per iteration",
           "command": "tools/pmc_selfplay.sh (separate --pmc passes; python3 bench.py --workload selfplay "
                      "--steps 40 --warmup 10)", "kernels": {}}
    for k in KERNELS:
        e = {}
        if k in du:
            e.update(du[k])
        if k in fe and k in wr:
            e["hbm_bytes_per_launch"] = fe[k]["FETCH_SIZE"] * 1024 * 2 + wr[k]["WRITE_SIZE"] * 1024
            if "avg_us" in e:
                e["hbm_GBps"] = e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e3)
        if k in sq:
            s = sq[k]
            w = max(s.get("SQ_WAVES", 1.0), 1.0)
            e["waves"] = s.get("SQ_WAVES")
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_MFMA"):
                if c in s:
                    e[c.lower().replace("sq_insts_", "") + "_per_wave"] = s[c] / w
            if "SQ_WAVE_CYCLES" in s and s["SQ_WAVE_CYCLES"]:
                e["wait_frac"] = s.get("SQ_WAIT_ANY", 0.0) / s["SQ_WAVE_CYCLES"]
        res["kernels"][k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
