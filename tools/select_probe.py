#!/usr/bin/env python3
"""k_select_lanes phase probes at config 3's steady state (diagnostic).

Runs bench.run_selfplay("config3") with the library named by SPLENDOR_AMD_LIB, built with
-DSELECT_PROBE=1, resets the probes right before the timed steps and prints the per-wave
average cycles of each phase over them: prologue (kept-root noise, resume, root scans),
descents (one NodeStat load per level), board staging, expansions (transition, fingerprint,
table lookup, end check) and leaf outputs, plus the slowest wave.
  SPLENDOR_AMD_LIB=$PWD/ablib/libprobe.so python3 tools/select_probe.py [--steps 1000]"""
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
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--prefill", type=int, default=6000)
    a = ap.parse_args()
    from splendor import _lib
    L = _lib.lib()
    has_sel = hasattr(L, "spl_diag_select_probe")   # (a -DBACKUP_PROBE=1 build has only that one)
    if has_sel:
        L.spl_diag_select_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 16)()

    bk = (ctypes.c_ulonglong * 16)()

    def reset(sp):
        torch.cuda.synchronize()
        if has_sel:
            L.spl_diag_select_probe(out, 1)
        if hasattr(L, "spl_diag_backup_probe"):
            L.spl_diag_backup_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
            L.spl_diag_backup_probe(bk, 1)
    dev = torch.device("cuda", 0)
    r = bench.run_selfplay("config3", 0, 1, dev, None, a.steps, 20, a.prefill, 0, 0x5EED,
                           stagger=min(4800, a.prefill), on_steady=reset)
    torch.cuda.synchronize()
    if has_sel:
        L.spl_diag_select_probe(out, 0)
    waves = max(int(out[5]), 1)
    names = ("prologue", "descents", "staging", "expansions", "leaf_outputs")
    res = {"steps": a.steps, "ms_per_iteration": r["elapsed"] / a.steps * 1e3, "waves": waves,
           "cycles_per_wave": {n: out[k] / waves for k, n in enumerate(names)},
           "total_cycles_per_wave": out[7] / waves, "max_wave_cycles": int(out[6]),
           "levels_deepest_lane_per_wave": out[8] / waves, "levels_per_lane": out[9] / (64 * waves),
           "most_levels": int(out[10]), "expansion_rounds_per_wave": out[11] / waves,
           "cycles_per_level_of_deepest_lane": out[1] / max(out[8], 1),
           "leaf_depth_max": r["tree"]["leaf_depth_max"]}
    if hasattr(L, "spl_diag_backup_probe"):
        L.spl_diag_backup_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        L.spl_diag_backup_probe(bk, 0)
        bw = max(int(bk[12]), 1)
        res["backup"] = {"waves": bw, "cycles_per_wave": {n: bk[k] / bw for k, n in enumerate(
            ("pass_a", "expansion_node_write", "pass_b_updates", "screen", "exact_levels", "writes_end",
             "expansion_alloc", "expansion_normalise", "expansion_sorted_run", "expansion_argmax"))},
            "exact_levels_per_wave": bk[13] / bw, "groups_per_wave": bk[14] / bw,
            "packed_groups_per_wave": bk[15] / bw}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
