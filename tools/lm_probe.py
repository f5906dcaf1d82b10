#!/usr/bin/env python3
"""k_leaf_mask per-workgroup timeline at config 3's steady state (diagnostic): the
library named by SPLENDOR_AMD_LIB built with -DLM_PROBE=1 records s_memrealtime (100 MHz) per
workgroup at entry, after the input / predicate / mask-word / pass-bit barriers and at exit of
the last launch; prints the spread of entry times, the workgroup lifetimes and the phases (us).
  SPLENDOR_AMD_LIB=$PWD/ablib/liblmprobe.so python3 tools/lm_probe.py [--steps 400]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--prefill", type=int, default=6000)
    a = ap.parse_args()
    from splendor import _lib
    L = _lib.lib()
    L.spl_diag_lm_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    dev = torch.device("cuda", 0)
    r = bench.run_selfplay("config3", 0, 1, dev, None, a.steps, 20, a.prefill, 0, 0x5EED,
                           stagger=min(4800, a.prefill))
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * (4096 * 8))()
    assert L.spl_diag_lm_probe(out) == 0
    t = np.frombuffer(out, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
    t = t[t[:, 0] > 0]
    us = 0.01                                     # 100 MHz ticks
    t0 = t[:, 0].min()
    pct = lambda x: {"p0": float(np.min(x) * us), "p50": float(np.median(x) * us),
                     "p90": float(np.percentile(x, 90) * us), "max": float(np.max(x) * us)}
    names = ("inputs", "predicates", "mask_words", "pass_bit", "stores")
    print(json.dumps({"ms_per_iteration": r["elapsed"] / a.steps * 1e3, "workgroups": int(len(t)),
                      "launch_span_us": float((t[:, 5].max() - t0) * us),
                      "entry_offset_us": pct(t[:, 0] - t0), "exit_offset_us": pct(t[:, 5] - t0),
                      "lifetime_us": pct(t[:, 5] - t[:, 0]),
                      "phases_us": {nm: pct(t[:, k + 1] - t[:, k]) for k, nm in enumerate(names)}}), flush=True)


if __name__ == "__main__":
    main()
