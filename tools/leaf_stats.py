import sys, os
sys.path.insert(0, "alphazero-general-ori_amd"); sys.path.insert(0, ".")
import numpy as np, torch
from bench import GENBU_ARGS
from splendor.env import SplendorEngine
from splendor.nnet import LeafEvaluator, random_net
from splendor.selfplay import SelfPlay
dev = torch.device("cuda", 0)
for n, B, sims, pre in ((2, 32768, 100, 3000), (4, 16384, 400, 20000)):
    eng = SplendorEngine(n, device=dev)
    ev = LeafEvaluator(eng, random_net(n, seed=0, device=dev), B, use_graph=False)
    sp = SelfPlay(eng, B, dict(GENBU_ARGS, numMCTSSims=sims), evaluator=ev)
    sp.reset()
    done = 0
    while done < pre:
        sp.run(2000, use_graph=True); done += 2000; sp.drain()
    fr = []
    for _ in range(50):
        sp.simulate()
        v = sp.leaf_valid.float().mean().item()
        h = sp.headers()
        fr.append((v, (h["leaf_kind"] == 2).mean(), (h["leaf_kind"] == 0).mean()))
        torch.cuda.synchronize()
        import splendor._lib as L
        L.check(sp.L.spl_mcts_commit(sp.h, sp.e._s()), "c")
    fr = np.array(fr)
    print(n, B, sims, "nn leaf frac", fr[:, 0].mean(), "terminal", fr[:, 1].mean(), "none", fr[:, 2].mean(), flush=True)
    del sp, ev; torch.cuda.empty_cache()
