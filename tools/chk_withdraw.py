#!/usr/bin/env python3
"""Diagnostic (bounds-checked library, SPLENDOR_AMD_LIB=ablib/libchk.so): the withdrawal
scenario of tests/test_selfplay_gpu.py::test_withdrawals_repeat_the_same_simulation at one
pool size (per-tree node slots, argv[1]), in chunks of 100 iterations, printing the
spl_diag_bounds counters (count, first value / site / tree, per-site counts) and events."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))
import torch  # noqa: E402


def main():
    from splendor import _lib
    from splendor.env import SplendorEngine
    from splendor.mcts import BatchedMCTS, HashEvaluator
    from splendor.selfplay import SelfPlay
    L = _lib.lib()
    L.spl_diag_bounds.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 68)()
    L.spl_diag_bounds(out, 1)
    per_tree = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    n, B, sims = 2, 64, 100
    nc = BatchedMCTS.default_node_cap(100)
    args = dict(numMCTSSims=sims, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5, forced_playouts=False,
                dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    e = SplendorEngine(n)
    sp = SelfPlay(e, B, args, evaluator=HashEvaluator(e, mode=1), dirichlet_noise=True, seed=11, out_cap=60000,
                  pool_nodes=B * per_tree, pool_edges=B * per_tree * BatchedMCTS.UNITS_PER_NODE, node_cap=nc,
                  edge_cap=32 * nc)
    sp.reset()
    for r in range(chunks):
        sp.run(100, use_graph=False)
        torch.cuda.synchronize()
        L.spl_diag_bounds(out, 0)
        st = sp.stats()
        print(json.dumps({"chunk": r, "violations": int(out[0]), "node": int(out[1]) >> 32,
                          "child": int(out[1]) & 0xFFFFFFFF, "value": int(out[1]), "site": int(out[2]),
                          "tree": int(out[3]), "sites": {k: int(out[4 + k]) for k in range(64) if out[4 + k]},
                          **{k: st[k] for k in ("withdrawals", "unexpanded", "prunes", "resets", "overflow",
                                                "collections")}}), flush=True)


if __name__ == "__main__":
    main()
