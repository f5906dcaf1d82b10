#!/usr/bin/env python3
"""Descent path reuse probe (development tool, GPU): config-3 self-play with the random-init
SplendorNNet (bench.py's workload) on a diagnostic build (MCTS_TIMING, tools/
libsplendor_diag.so); reports per simulation the levels descended and how many of them
repeat the previous simulation's path (node and edge) from the root — the share a
speculative prefetch of the previous path could serve.

  (cd alphazero-general-ori_amd && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC \
      -ffp-contract=off -DMCTS_TIMING=1 -shared -o ../tools/libsplendor_diag.so \
      csrc/splendor_env.hip csrc/mcts.hip csrc/nnet.hip)
  SPLENDOR_AMD_LIB=tools/libsplendor_diag.so python tools/select_reuse.py [warm] [iters]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    from splendor import _lib
    from splendor.env import SplendorEngine
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.selfplay import SelfPlay
    from bench import GENBU_ARGS
    L = _lib.lib()
    L.spl_diag_select_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
    B = 32768
    eng = SplendorEngine(2)
    ev = LeafEvaluator(eng, random_net(2, seed=0), B, use_graph=False)
    sp = SelfPlay(eng, B, dict(GENBU_ARGS, numMCTSSims=100), evaluator=ev, dirichlet_noise=True)
    sp.reset()
    buf = (ctypes.c_ulonglong * 24)()
    for k, n in ((0, warm), (1, iters)):
        sp.run(n, use_graph=True)
        torch.cuda.synchronize()
        L.spl_diag_select_timing(buf, 1)
        if k == 1:
            h = list(buf)
            sims = h[21]
            print(f"{iters} iterations: {h[23] / sims:.2f} levels per simulation, "
                  f"{h[22] / sims:.2f} of them repeat the previous simulation's path", flush=True)
        sp.drain(allow_drops=True)


if __name__ == "__main__":
    main()
