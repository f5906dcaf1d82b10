#!/usr/bin/env python3
"""Tree-pool sizing probe (development tool, GPU): runs batched self-play with generous
per-tree caps and reports, every --every iterations, the node / edge counts of the trees
(max, 99.9th / 99th / 50th percentile) and per-node edge averages, so the per-tree caps of
spl_mcts_create can be set from measurement.

  python tools/tree_sizes.py --players 2 --boards 1024 --sims 1600 --iters 60000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--boards", type=int, default=1024)
    ap.add_argument("--sims", type=int, default=1600)
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--every", type=int, default=2000)
    ap.add_argument("--node-cap", type=int, default=0)
    ap.add_argument("--edge-cap", type=int, default=0)
    ap.add_argument("--out", default="")
    ap.add_argument("--default-caps", action="store_true", help="SelfPlay's own default caps")
    a = ap.parse_args()
    from splendor.env import SplendorEngine
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.selfplay import SelfPlay
    sys.path.insert(0, ROOT)
    from bench import GENBU_ARGS
    dev = torch.device("cuda", 0)
    eng = SplendorEngine(a.players, device=dev)
    net = random_net(a.players, seed=0, device=dev)
    ev = LeafEvaluator(eng, net, a.boards, use_graph=False)
    ncap = a.node_cap or 8 * a.sims + 64
    ecap = a.edge_cap or 48 * ncap
    caps = {} if a.default_caps else dict(node_cap=ncap, edge_cap=ecap)
    sp = SelfPlay(eng, a.boards, dict(GENBU_ARGS, numMCTSSims=a.sims), evaluator=ev, dirichlet_noise=True,
                  out_cap=64 * a.boards, **caps)
    ncap, ecap = sp.cfg.node_cap, sp.cfg.edge_cap
    sp.reset()
    rows = []
    t0 = time.perf_counter()
    done = 0
    while done < a.iters:
        k = min(a.every, a.iters - done)
        sp.run(k, use_graph=True)
        done += k
        h = sp.headers()
        sp.drain()
        nc, ec = h["node_count"].astype(np.int64), h["edge_count"].astype(np.int64)
        ts = sp.tree_sizes().astype(np.int64)
        ln, le = ts[:, 2], ts[:, 3]
        live = {"live_nodes": [int(ln.max()), int(np.percentile(ln, 99.9)), int(np.percentile(ln, 99)),
                               int(np.median(ln)), round(float(ln.mean()), 1)],
                "live_edges": [int(le.max()), int(np.percentile(le, 99.9)), int(np.percentile(le, 99)),
                               int(np.median(le)), round(float(le.mean()), 1)]}
        r = {"iter": done, "s": round(time.perf_counter() - t0, 1), "games_done": int(h["games_done"].sum()),
             "overflow": int((h["overflow"] != 0).sum()),
             "nodes": [int(nc.max()), int(np.percentile(nc, 99.9)), int(np.percentile(nc, 99)), int(np.median(nc))],
             "edges": [int(ec.max()), int(np.percentile(ec, 99.9)), int(np.percentile(ec, 99)), int(np.median(ec))],
             "nodes_mean": round(float(nc.mean()), 1), "edges_mean": round(float(ec.mean()), 1),
             "nodes_deciles": [int(x) for x in np.percentile(nc, range(10, 100, 10))],
             "edges_deciles": [int(x) for x in np.percentile(ec, range(10, 100, 10))],
             "events": sp.capacity_events(h), **live,
             "edges_per_node_max": round(float((ec / np.maximum(nc, 1)).max()), 1),
             "edges_per_node_mean": round(float(ec.sum() / max(nc.sum(), 1)), 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    res = {"players": a.players, "boards": a.boards, "sims": a.sims, "node_cap": ncap, "edge_cap": ecap,
           "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
