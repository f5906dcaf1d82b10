#!/usr/bin/env python3
"""k_rollout launch-size sweep (development tool, GPU): average kernel time of one launch of
K moves over 32,768 boards (HIP events, back-to-back launches) for several K, and the
fitted fixed cost per launch + cost per move.

  python tools/rollout_sweep.py [--players 2] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--boards", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ks", default="1,2,5,10,20,50,100,200")
    a = ap.parse_args()
    from splendor.env import RolloutBatch, SplendorEngine
    e = SplendorEngine(a.players, device="cuda:0")
    rb = RolloutBatch(e, a.boards, seed=0x5EED)
    rb.run(100)
    rows = []
    for K in [int(x) for x in a.ks.split(",")]:
        out = rb.run(K)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            rb.run(K, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        rows.append({"K": K, "us_per_launch": round(us, 2), "us_per_move": round(us / K, 3),
                     "board_steps_per_s": a.boards * K / (us * 1e-6)})
        print(json.dumps(rows[-1]), flush=True)
    ks = np.array([r["K"] for r in rows], float)
    us = np.array([r["us_per_launch"] for r in rows])
    fit = np.polyfit(ks, us, 1)
    print(json.dumps({"fit_us_per_move": fit[0], "fit_us_fixed": fit[1]}))


if __name__ == "__main__":
    main()
