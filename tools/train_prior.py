#!/usr/bin/env python3
"""A trained 2-player prior for the benchmark's trained-prior regime: Coach.learn
(Coach.py:102-164, splendor/coach.py) on device self-play at genbu.pt's search arguments, from a
seeded random-init SplendorNNet, for a few iterations: numEps games per iteration on as many
concurrent trees, training on the example history (GenericNNetWrapper.train's losses and
schedule, larger batches), the BatchedArena gate against the previous weights. Writes the
accepted weights as a plain state_dict checkpoint ({"state_dict": ...}, weights-only loadable)
and one JSON line per iteration (losses, arena result, self-play figures) to stdout:
    python3 tools/train_prior.py OUT.pt [iterations] [games]
bench.py --net OUT.pt then runs the headline on these weights."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

from splendor.NNet import NNetWrapper  # noqa: E402
from splendor.SplendorGame import SplendorGame  # noqa: E402
from splendor.coach import Coach  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trained_2p.pt"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
games = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
# (Coach.learn's checkpoints and example history stay out of gpurun_out: only OUT is kept)
folder = os.path.join(os.environ.get("TMPDIR", "/tmp"), "train_prior_ckpt")
g = SplendorGame(2)
torch.manual_seed(0)
nn = NNetWrapper(g, dict(epochs=2, batch_size=512, learn_rate=1e-3, dropout=0.3), seed=0)
args = dict(numMCTSSims=100, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5, forced_playouts=False,
            dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10, numIters=1, numEps=games,
            numItersHistory=3, arenaCompare=256, updateThreshold=0.55, checkpoint=folder)
coach = Coach(g, nn, args, batch=games, seed=0x7A11)
last = {}
orig_train = nn.train


def train(examples, **kw):
    r = orig_train(examples, **kw)
    last["losses"] = r
    last["examples"] = len(examples)
    return r


nn.train = train
pnet = NNetWrapper(g, dict(nn.args), device=nn.device)
accepted = 0
for i in range(1, iters + 1):
    t0 = time.perf_counter()
    (nw, pw, dr, ok), = coach.learn(pnet=pnet)
    accepted += bool(ok)
    st = coach.sp.stats()
    print(json.dumps({"iteration": i, "seconds": time.perf_counter() - t0, "examples": last.get("examples"),
                      "losses": {k: float(v) for k, v in (last.get("losses") or {}).items()},
                      "arena_new_prev_draws": [nw, pw, dr], "accepted": bool(ok),
                      "selfplay_leaf_depth_now": st["leaf_depth_now"]}), flush=True)
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
torch.save({"state_dict": nn.nnet.state_dict(), "iterations": iters, "accepted": accepted}, out)
print(json.dumps({"saved": out, "iterations": iters, "accepted": accepted}), flush=True)
