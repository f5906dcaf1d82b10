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

KERNELS = ("k_select", "k_leaf_mask", "k_nn_forward", "k_backup", "k_commit", "k_gc")



def _kname(k):
    """k_select_lanes (lane per tree) is the select kernel, k_backup_h (two trees per wave) the
    backup kernel: reported as k_select / k_backup."""
    return {"k_select_lanes": "k_select", "k_backup_h": "k_backup"}.get(k, k)

def per_kernel(d, last=None):
    """Counter averages per dispatch of each kernel, over its last `last` dispatches."""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"k_\w+", r.get("Kernel_Name", ""))
            if not m or _kname(m.group(0)) not in KERNELS:
                continue
            k, disp = _kname(m.group(0)), int(r["Dispatch_Id"])
            acc.setdefault(k, {}).setdefault(disp, {})
            c = r["Counter_Name"]
            acc[k][disp][c] = acc[k][disp].get(c, 0.0) + float(r["Counter_Value"])
    out = {}
    for k, disps in acc.items():
        ids = sorted(disps)[-last:] if last else sorted(disps)
        names = {c for i in ids for c in disps[i]}
        out[k] = {c: sum(disps[i].get(c, 0.0) for i in ids) / len(ids) for c in names}
    return out


def durations(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"k_\w+", r["Name"])
            if m and _kname(m.group(0)) in KERNELS:
                out[_kname(m.group(0))] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def main():
    root, rnd = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else None
    warm = int(sys.argv[4]) if len(sys.argv) > 4 else None
    fe, wr, sq, sq2, mem, ea = (per_kernel(os.path.join(root, x), steps)
                                for x in ("fetch", "write", "sq", "sq2", "mem", "ea"))
    du = durations(os.path.join(root, "trace"))
    res = {"round": rnd, "workload": "config 3: 32768 self-play games, numMCTSSims=100 (genbu args), "
           "one select/network/backup/commit per iteration, steady state",
           "command": f"tools/pmc_selfplay.sh (separate --pmc passes; python3 bench.py --workload selfplay "
                      f"--steps {steps} --warmup {warm}); counters averaged over each kernel's last {steps} "
                      f"dispatches; durations: kernel trace over the whole run",
           "kernels": {}}
    for k in KERNELS:
        e = {}
        if k in du:
            e.update(du[k])
        if k in fe and k in wr:
            e["hbm_bytes_per_launch"] = fe[k]["FETCH_SIZE"] * 1024 * 2 + wr[k]["WRITE_SIZE"] * 1024
            if "avg_us" in e:
                e["hbm_GBps"] = e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e3)
        s = {**sq.get(k, {}), **sq2.get(k, {}), **mem.get(k, {}), **ea.get(k, {})}
        if "TCC_EA0_RDREQ_sum" in s:
            # memory-side read requests by size (MI355X_MICROARCH.md: FETCH_SIZE = RDREQ x 64 B,
            # exact only for 128-B streaming reads); random small reads are sized per request
            n, n32, n128 = s["TCC_EA0_RDREQ_sum"], s.get("TCC_EA0_RDREQ_32B_sum", 0.0), s.get("TCC_EA0_RDREQ_128B_sum", 0.0)
            e["read_bytes_by_request_size"] = 32 * n32 + 64 * max(n - n32 - n128, 0.0) + 128 * n128
            if k in wr:
                e["hbm_bytes_per_launch_by_request_size"] = e["read_bytes_by_request_size"] + wr[k]["WRITE_SIZE"] * 1024
        if s:
            w = max(s.get("SQ_WAVES", 1.0), 1.0)
            e["waves"] = s.get("SQ_WAVES")
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_LDS", "SQ_INSTS_MFMA"):
                if c in s:
                    e[c.lower().replace("sq_insts_", "") + "_per_wave"] = s[c] / w
            wc = s.get("SQ_WAVE_CYCLES")
            if wc:
                e["wait_frac"] = s.get("SQ_WAIT_ANY", 0.0) / wc
                e["wait_inst_frac"] = s.get("SQ_WAIT_INST_ANY", 0.0) / wc
                e["active_inst_frac"] = s.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
                e["wave_cycles_per_wave"] = wc / w
            if s.get("SQ_INSTS_VMEM_RD") and "SQ_INST_LEVEL_VMEM" in s:
                e["vmem_latency_cycles"] = s["SQ_INST_LEVEL_VMEM"] / (s["SQ_INSTS_VMEM_RD"] + s.get("SQ_INSTS_VMEM_WR", 0.0))
            if s.get("TCP_TCC_READ_REQ_sum"):
                e["l2_read_latency_cycles"] = s.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / s["TCP_TCC_READ_REQ_sum"]
                e["l2_read_requests"] = s["TCP_TCC_READ_REQ_sum"]
            if s.get("TCC_HIT_sum") is not None and s.get("TCC_MISS_sum") is not None:
                e["l2_hit_rate"] = s["TCC_HIT_sum"] / max(s["TCC_HIT_sum"] + s["TCC_MISS_sum"], 1.0)
            tm, th = s.get("TCP_UTCL1_TRANSLATION_MISS_sum"), s.get("TCP_UTCL1_TRANSLATION_HIT_sum")
            if tm is not None and th is not None:
                e["utcl1_miss_rate"] = tm / max(tm + th, 1.0)
            e["raw"] = s
        res["kernels"][k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
