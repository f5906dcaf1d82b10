#!/usr/bin/env python3
"""k_nn_forward per-layer cycle probes over a full batch (diagnostic): the
library named by SPLENDOR_AMD_LIB built with -DNN_PROBE=1 (wave 0 of every workgroup stamps
each layer boundary), B = 32,768 leaves of mid-game positions, a seeded random-init network;
prints the average cycles per workgroup of each stage.
  SPLENDOR_AMD_LIB=$PWD/ablib/libnnprobe.so python3 tools/nn_probe.py [B] [players]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

from splendor import _lib  # noqa: E402
from splendor.env import RolloutBatch, SplendorEngine  # noqa: E402
from splendor.nnet import LeafEvaluator, random_net  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
eng = SplendorEngine(N, device=dev)
rb = RolloutBatch(eng, B, seed=7)
rb.run(30)
state = eng.canonical(rb.state, rb.player)
mask = eng.valid_moves(state)
ev = LeafEvaluator(eng, random_net(N, seed=0, device=dev), B, use_graph=False)
L = _lib.lib()
L.spl_diag_nn_probe.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
out = (ctypes.c_ulonglong * 16)()
for _ in range(5):
    ev(state, mask)
torch.cuda.synchronize(dev)
L.spl_diag_nn_probe(out, 1)
for _ in range(20):
    ev(state, mask)
torch.cuda.synchronize(dev)
L.spl_diag_nn_probe(out, 0)
wg = max(int(out[15]), 1)
names = ("input", "dense2d_1", "dense2d_1[3]", "partialgpool_1", "dense2d_3+flatten", "dense1d_4", "pgp4..pgp5",
         "heads_PI0_V0", "PI1_V1", "softmax")
per = {n: out[k] / wg for k, n in enumerate(names)}
print(json.dumps({"B": B, "players": N, "workgroups": wg, "cycles_per_workgroup": per,
                  "total": sum(per.values())}, indent=1))
