#!/usr/bin/env python3
"""Pool planning probe (development tool, GPU): the per-tree caps, node-board choice and
arena bytes BatchedMCTS._caps plans for BASELINE configs 3-5 on this device.

  python tools/plan_caps.py
"""
import sys, os
sys.path.insert(0, os.path.join(os.getcwd(), "alphazero-general-ori_amd"))
import torch
from splendor.env import SplendorEngine
from splendor.selfplay import SelfPlay
from splendor.mcts import HashEvaluator
GENBU = dict(cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5, forced_playouts=False,
             dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
for n, B, sims in ((2, 32768, 100), (2, 32768, 1600), (4, 16384, 400)):
    e = SplendorEngine(n)
    sp = SelfPlay(e, B, dict(GENBU, numMCTSSims=sims), evaluator=HashEvaluator(e))
    print(n, B, sims, "node_cap", sp.cfg.node_cap, "edge_cap", sp.cfg.edge_cap, "node_boards", sp.cfg.node_boards,
          "GiB", round(sp.device_bytes / 2**30, 1), flush=True)
    del sp; torch.cuda.empty_cache()
