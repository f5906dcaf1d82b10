#!/usr/bin/env python3
"""k_nn_forward on the search's NN-leaf list (spl_nn_forward_indexed) at config 3's shape:
B = 32,768 trees of which FRAC have an NN leaf (0.69 at config 3), listed as the library's ABI
expects — ABI <= 10: one compact list and one count; ABI 11: per 64-tree segment — for the
same leaves; HIP events over 50 launches after 10 warm-up. The library is loaded directly
(SPLENDOR_AMD_LIB or the in-tree one), so an older ABI can be timed beside the current one:
    SPLENDOR_AMD_LIB=... python3 tools/nn_indexed_time.py [FRAC]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

from splendor.env import RolloutBatch, SplendorEngine  # noqa: E402
from splendor.nnet import FoldedNet, pack_weights, random_net  # noqa: E402

FRAC = float(sys.argv[1]) if len(sys.argv) > 1 else 0.69
B, N, WARM, ITERS = 32768, 2, 10, 50
path = os.environ.get("SPLENDOR_AMD_LIB") or os.path.join(ROOT, "alphazero-general-ori_amd", "libsplendor_amd.so")
L = C.CDLL(path)
abi = L.spl_abi_version()
vp = C.c_void_p
L.spl_nn_forward_indexed.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
dev = torch.device("cuda", 0)
eng = SplendorEngine(N, device=dev)
rb = RolloutBatch(eng, B, seed=7)
rb.run(30)
state = eng.canonical(rb.state, rb.player).contiguous()
mask = eng.valid_moves(state).contiguous()
w = pack_weights(FoldedNet(random_net(N, seed=0, device=dev)).to(dev).eval(), N)
rng = np.random.default_rng(3)
valid = rng.random(B) < FRAC
rows = np.nonzero(valid)[0].astype(np.int32)
if abi >= 11:
    idx = np.zeros(B, np.int32)
    cnt = np.zeros((B + 63) // 64, np.int32)
    for j in range(len(cnt)):
        r = rows[(rows >= 64 * j) & (rows < 64 * j + 64)]
        idx[64 * j:64 * j + len(r)] = r
        cnt[j] = len(r)
else:
    idx = np.zeros(B, np.int32)
    idx[:len(rows)] = rows if os.environ.get("NN_ORDER") == "sorted" else rng.permutation(rows)
    cnt = np.array([len(rows)], np.int32)
idx_t, cnt_t = torch.from_numpy(idx).to(dev), torch.from_numpy(cnt).to(dev)
pi = torch.zeros(B, 409, device=dev)
v = torch.zeros(B, N, device=dev)
s = torch.cuda.current_stream(dev)
p = lambda t: C.c_void_p(t.data_ptr())


def launch():
    assert L.spl_nn_forward_indexed(N, B, p(state), p(mask), p(idx_t), p(cnt_t), p(w), p(pi), p(v),
                                    C.c_void_p(s.cuda_stream)) == 0


for _ in range(WARM):
    launch()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(dev)
e0.record()
for _ in range(ITERS):
    launch()
e1.record()
torch.cuda.synchronize(dev)
print(json.dumps({"abi": abi, "order": os.environ.get("NN_ORDER", "random"), "lib": path, "leaves": int(len(rows)), "tiles": -(-len(rows) // 32),
                  "us_per_launch": e0.elapsed_time(e1) / ITERS * 1e3,
                  "pi_checksum": float(pi[torch.from_numpy(rows).to(dev).long()].double().sum())}), flush=True)
