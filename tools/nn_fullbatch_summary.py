#!/usr/bin/env python3
"""Summarise tools/nn_fullbatch.sh: k_nn_forward<2> over a full batch of 32,768 leaves —
rocprofv3 average duration, HBM bytes per launch (FETCH_SIZE KB x1024 x2 gfx950 correction
+ WRITE_SIZE KB x1024, as tools/pmc_selfplay_summary.py), the bf16 MFMA FLOPs it executes
against the dense bf16 peak and the instruction mix's MFMA floor (bench.nn_mix_ceiling_us),
and the f32-equivalent rate (1.19 MFLOP per leaf, bench.nn_flops_per_eval) against the f32
MFMA peak."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pmc_selfplay_summary import durations, per_kernel  # noqa: E402
import bench  # noqa: E402

d, rnd = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r03"
B, FLOP_PER_LEAF, PEAK = 32768, 2 * 595328, 157.3
dur = durations(os.path.join(d, "trace")).get("k_nn_forward", {})
fe = per_kernel(os.path.join(d, "FETCH_SIZE")).get("k_nn_forward", {})
wr = per_kernel(os.path.join(d, "WRITE_SIZE")).get("k_nn_forward", {})
hbm = fe["FETCH_SIZE"] * 1024 * 2 + wr["WRITE_SIZE"] * 1024 if fe and wr else None
us = dur.get("avg_us")
tf = FLOP_PER_LEAF * B / (us * 1e-6) / 1e12 if us else None
ceil_us, xfl = bench.nn_mix_ceiling_us(2, B)
print(json.dumps({"round": rnd, "kernel": "k_nn_forward<2>", "leaves_per_launch": B,
                  "command": "tools/nn_fullbatch.sh (python3 tools/nn_fullbatch.py: 10 + 50 launches)",
                  "calls": dur.get("calls"), "avg_us": us, "hbm_bytes_per_launch": hbm,
                  "executed_bf16_flop_per_launch": xfl,
                  "executed_bf16_tflops": xfl / (us * 1e-6) / 1e12 if us else None,
                  "frac_bf16_mfma_peak": xfl / (us * 1e-6) / 1e12 / bench.BF16_MFMA_PEAK if us else None,
                  "mix_ceiling_us": ceil_us, "frac_of_mix_ceiling": ceil_us / us if us else None,
                  "flop_per_launch": FLOP_PER_LEAF * B, "tflops_f32_equivalent": tf,
                  "frac_fp32_mfma_peak": tf / PEAK if tf else None},
                 indent=1))
