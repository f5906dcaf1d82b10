#!/usr/bin/env python3
"""compact_tree per-phase cycle probes at config 3's steady state (diagnostic):
the library named by SPLENDOR_AMD_LIB built with -DGC_PROBE=1; resets the probes right before
the timed steps and prints the average cycles per collection of each phase and the slowest
collection (its cycles, units and nodes).
  SPLENDOR_AMD_LIB=$PWD/ablib/libgcprobe.so python3 tools/gc_probe.py [--steps 2000]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--prefill", type=int, default=6000)
    a = ap.parse_args()
    from splendor import _lib
    L = _lib.lib()
    L.spl_diag_gc_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 24)()

    def reset(sp):
        torch.cuda.synchronize()
        L.spl_diag_gc_probe(out, 1)
    dev = torch.device("cuda", 0)
    r = bench.run_selfplay("config3", 0, 1, dev, None, a.steps, 20, a.prefill, 0, 0x5EED,
                           stagger=min(4800, a.prefill), on_steady=reset)
    torch.cuda.synchronize()
    L.spl_diag_gc_probe(out, 0)
    n = max(int(out[8]), 1)
    names = ("keep_remap", "sizes_packing", "node_records", "links_owner_map", "unit_staging",
             "writeback_boards", "table_pages")
    print(json.dumps({"steps": a.steps, "ms_per_iteration": r["elapsed"] / a.steps * 1e3, "collections": n,
                      "cycles_per_collection": {nm: out[k] / n for k, nm in enumerate(names)},
                      "total_cycles_per_collection": out[9] / n,
                      "slowest": {"cycles": int(out[10]), "units": int(out[11]), "kept_nodes": int(out[12]),
                                  "nodes_before": int(out[13]),
                                  "phases": {nm: int(out[16 + k]) for k, nm in enumerate(names)}}}), flush=True)


if __name__ == "__main__":
    main()
