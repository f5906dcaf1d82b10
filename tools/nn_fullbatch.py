#!/usr/bin/env python3
"""k_nn_forward alone over a full batch (the headline roofline's kernel and unit): B leaf
boards = B freshly dealt games plus RANDOM_MOVES random plies each (positions of every
stage), their legality masks, a seeded random-init SplendorNNet; WARM untimed launches, then
ITERS launches timed with HIP events on the launch stream. Run it under rocprofv3
(--kernel-trace --stats, or --pmc FETCH_SIZE / WRITE_SIZE with a k_nn_forward filter) for the
kernel's own duration and HBM bytes per launch at the same batch:
    python3 tools/nn_fullbatch.py [B] [players]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

from splendor.env import RolloutBatch, SplendorEngine  # noqa: E402
from splendor.nnet import LeafEvaluator, random_net  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2
WARM, ITERS, RANDOM_MOVES = 10, 50, 30
dev = torch.device("cuda", 0)
eng = SplendorEngine(N, device=dev)
rb = RolloutBatch(eng, B, seed=7)
rb.run(RANDOM_MOVES)
state = eng.canonical(rb.state, rb.player)
mask = eng.valid_moves(state)
ev = LeafEvaluator(eng, random_net(N, seed=0, device=dev), B, use_graph=False)
for _ in range(WARM):
    ev(state, mask)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(dev)
e0.record()
for _ in range(ITERS):
    ev(state, mask)
e1.record()
torch.cuda.synchronize(dev)
us = e0.elapsed_time(e1) / ITERS * 1e3
print(f"k_nn_forward<{N}> B={B}: {us:.1f} us per launch (HIP events, {ITERS} launches)")
