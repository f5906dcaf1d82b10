#!/usr/bin/env python3
"""Per-kernel mean / max duration over the last N dispatches of a rocprofv3 kernel trace
(usage: tools/trace_split.py gpurun_out/qprof/sp_kernel_trace.csv [N])."""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
per = defaultdict(list)
for r in csv.DictReader(open(path)):
    m = re.search(r'(k_\w+)', r['Kernel_Name'])
    k = m.group(1) if m else r['Kernel_Name'][:30]
    per[k].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = 0.0
# launches per iteration of each kernel, relative to k_select_lanes (one per iteration): k_gc ran
# twice per iteration until the self-play backup deferred its collection (SPL_BACKUP_DEFER_GC)
ref = len(per.get('k_select_lanes', [])) or 1
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1][-n:])):
    if len(v) < 100:
        continue
    ratio = max(1, round(len(v) / ref))
    last = v[-ratio * n:]
    per_it = sum(last) / n / 1000
    tot += per_it
    print(f"{k:16s} calls={len(v):6d}  mean={sum(last) / len(last) / 1000:7.1f} us  max={max(last) / 1000:7.1f} us  "
          f"per iteration={per_it:7.1f} us")
print(f"{'sum':16s} {tot:.1f} us per iteration")
