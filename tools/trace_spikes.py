#!/usr/bin/env python3
"""Latency spikes in a rocprofv3 kernel trace of the self-play loop (VERDICT r04 Next #7).

For each self-play kernel: the launch-time distribution over the last N iterations (p50, p99,
max) and the slowest launches with their iteration index (the k_commit launches number the
iterations) and what ran around them — whether the iteration was a commit iteration (one in
20 at config 3: the search boundary), how long that iteration's k_gc launches took, and the
network launch of the same iteration.

usage: tools/trace_spikes.py <kernel_trace.csv> [N iterations] [top K]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rows = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if not m:
            continue
        k = m.group(1)
        k = {"k_select_lanes": "k_select", "k_backup_h": "k_backup"}.get(k, k)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # iterations: a k_select launch opens one
    it, per = -1, []
    for s, e, k in rows:
        if k == "k_select":
            it += 1
            per.append(defaultdict(list))
        if it >= 0:
            per[it][k].append((e - s) / 1e3)
    per = per[-n:]
    out = {"iterations": len(per), "kernels": {}}
    for k in ("k_select", "k_leaf_mask", "k_nn_forward", "k_backup", "k_gc", "k_commit"):
        d = sorted(x for p in per for x in p.get(k, []))
        if not d:
            continue
        q = lambda f: d[min(len(d) - 1, int(f * len(d)))]
        worst = sorted(((max(p[k]), i) for i, p in enumerate(per) if p.get(k)), reverse=True)[:top]
        out["kernels"][k] = {
            "launches": len(d), "mean_us": sum(d) / len(d), "p50_us": q(0.5), "p99_us": q(0.99), "max_us": d[-1],
            "slowest": [{"iteration": i, "us": round(v, 1),
                         "commit_iteration": bool(per[i].get("k_commit")) and max(per[i]["k_commit"]) > 30,
                         "gc_us": [round(x, 1) for x in per[i].get("k_gc", [])],
                         "nn_us": [round(x, 1) for x in per[i].get("k_nn_forward", [])],
                         "commit_us": [round(x, 1) for x in per[i].get("k_commit", [])]}
                        for v, i in worst]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
