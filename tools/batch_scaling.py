#!/usr/bin/env python3
"""Diagnostic: the config-3 self-play step at a given number of games (argv[1], default
32768) — bench.run_selfplay with config 3's batch overridden — to see how each kernel's time
scales with the batch (run under rocprofv3 --kernel-trace; tools/trace_split.py on the trace):
    python3 tools/batch_scaling.py B"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
n, _, sims = bench.CONFIGS["config3"]
bench.CONFIGS["config3"] = (n, B, sims)
r = bench.run_selfplay("config3", 0, 1, torch.device("cuda", 0), None, 1000, 100, 6000, 0, 0x5EED, stagger=4800)
print(f"B={B}: {r['elapsed'] / 1000 * 1e3:.3f} ms per iteration, {B * 1000 / r['elapsed'] / 1e6:.2f} M sims/s", flush=True)
