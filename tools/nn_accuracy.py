#!/usr/bin/env python3
"""k_nn_forward's error against a float64 evaluation of the same folded network (diagnostic):
B positions of every game stage (fresh deals + 30 random plies), a seeded random-init
SplendorNNet; the loaded library's fused kernel (SPLENDOR_AMD_LIB picks the build: the
product, or ablib/libsplit.so with NN_SPLIT=1) and PyTorch fp32 on the CPU (the reference's
own precision and path) are both compared with FoldedNet in float64. Prints one JSON line:
    python3 tools/nn_accuracy.py [B] [players] [tag]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

from splendor.env import RolloutBatch, SplendorEngine  # noqa: E402
from splendor.nnet import FoldedNet, LeafEvaluator, random_net  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2
TAG = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(os.environ.get("SPLENDOR_AMD_LIB", "product"))
dev = torch.device("cuda", 0)
eng = SplendorEngine(N, device=dev)
rb = RolloutBatch(eng, B, seed=11)
rb.run(30)
state = eng.canonical(rb.state, rb.player)
mask = eng.valid_moves(state)
net = random_net(N, seed=3, device=dev)
ev = LeafEvaluator(eng, net, B, use_graph=False)
pi, v = (t.double().cpu() for t in ev(state, mask))
ev._convert(state, mask)
x, valid = ev.x.cpu(), ev.valid.cpu()
with torch.no_grad():
    f64 = FoldedNet(net.cpu()).double().eval()
    pi64, v64 = f64(x.double(), valid, transposed=True)
    f32 = FoldedNet(net.cpu()).float().eval()
    pi32, v32 = (t.double() for t in f32(x, valid, transposed=True))


def err(a, ref):
    d = (a - ref).abs()
    big = ref.abs() > 1e-3
    return {"max_abs": float(d.max()), "mean_abs": float(d.mean()),
            "max_rel_gt1e-3": float((d[big] / ref.abs()[big]).max()) if big.any() else 0.0}


print(json.dumps({"lib": TAG, "B": B, "players": N,
                  "kernel": {"pi": err(pi, pi64), "v": err(v, v64)},
                  "torch_cpu_fp32": {"pi": err(pi32, pi64), "v": err(v32, v64)}}), flush=True)
