#!/usr/bin/env python3
"""Diagnostic (bounds-checked library, SPLENDOR_AMD_LIB=ablib/libchk.so): the capacity-pressure
self-play of tests/test_configs_gpu.py::test_capacity_pressure_is_graceful, then the bounds /
link-consistency counter of spl_diag_bounds: [count, first value, site, tree] + per-site counts."""
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
    from splendor.mcts import HashEvaluator
    from splendor.selfplay import SelfPlay
    L = _lib.lib()
    L.spl_diag_bounds.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 68)()
    L.spl_diag_bounds(out, 1)
    genbu = dict(cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5, forced_playouts=False,
                 dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    n, B, sims = 2, 256, 64
    e = SplendorEngine(n)
    sp = SelfPlay(e, B, dict(genbu, numMCTSSims=sims), evaluator=HashEvaluator(e), dirichlet_noise=True,
                  seed=0x5EED, node_cap=96, edge_cap=96 * 24)
    sp.reset()
    for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
        sp.run(400, use_graph=True)
        sp.drain()
        torch.cuda.synchronize()
        L.spl_diag_bounds(out, 0)
        st = sp.stats()
        print(json.dumps({"round": r, "violations": int(out[0]), "value": int(out[1]), "node": int(out[1]) >> 32,
                          "child": int(out[1]) & 0xFFFFFFFF, "site": int(out[2]), "tree": int(out[3]),
                          "sites": {k: int(out[4 + k]) for k in range(64) if out[4 + k]},
                          "overflow": st["overflow"], "prunes": st["prunes"], "resets": st["resets"],
                          "withdrawals": st["withdrawals"], "unexpanded": st["unexpanded"]}), flush=True)


if __name__ == "__main__":
    main()
