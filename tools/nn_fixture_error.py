#!/usr/bin/env python3
"""The fused network's error against the reference network's recorded outputs
(tests/golden/nnet_{2,3,4}p.npz: the reference SplendorNNet with closed-form weights), for the
library SPLENDOR_AMD_LIB loads (the product, or ablib/libf32.so built with NN_SPLIT=0):
max |pi - pi_ref|, max relative error where pi_ref > 1e-6, max |v - v_ref|. One JSON line.
    python3 tools/nn_fixture_error.py [tag]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_nnet import GOLD, _pack_mask, deterministic_weights  # noqa: E402

from splendor.nnet import FusedNet, SplendorNNet  # noqa: E402

out = {"lib": sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("SPLENDOR_AMD_LIB", "product"))}
for n in (2, 3, 4):
    with np.load(os.path.join(GOLD, f"nnet_{n}p.npz")) as z:
        g = {k: z[k] for k in z.files}
    net = SplendorNNet(n)
    net.load_state_dict(deterministic_weights(net.state_dict()))
    fused = FusedNet(net.cuda().eval(), n, "cuda")
    boards = torch.from_numpy(np.ascontiguousarray(g["boards"].astype(np.int8))).cuda()
    mask = torch.from_numpy(_pack_mask(g["valid"])).cuda()
    pi, v = fused(boards, mask)
    pi, v = pi.double().cpu().numpy(), v.double().cpu().numpy()
    ref = np.exp(g["log_pi"].astype(np.float64)) * g["valid"]
    d = np.abs(pi - ref)
    big = ref > 1e-6
    out[f"{n}p"] = {"pi_max_abs": float(d.max()), "pi_max_rel": float((d[big] / ref[big]).max()),
                    "v_max_abs": float(np.abs(v - g["v"].astype(np.float64)).max()), "rows": int(ref.shape[0])}
print(json.dumps(out), flush=True)
