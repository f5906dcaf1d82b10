"""SplendorNNet re-implementation vs the reference network (golden outputs recorded by
make_golden.py from the reference's SplendorNNet with closed-form weights). fp32 on CPU;
tolerance 1e-5 absolute on log-probabilities/values (reduction-order differences only)."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def deterministic_weights(state_dict):
    out = {}
    for k, name in enumerate(sorted(state_dict)):
        t = state_dict[name]
        if not t.is_floating_point():
            out[name] = t.clone()
            continue
        i = torch.arange(t.numel(), dtype=torch.float64)
        u = torch.remainder(i * 0.6180339887498949 + 0.1234 * (k + 1), 1.0)
        if name.endswith("running_var"):
            v = 0.5 + u
        elif name.endswith("lowvalue"):
            v = torch.full_like(u, -1e8)
        else:
            v = (u - 0.5) * (0.3 if name.endswith("weight") else 0.1)
        out[name] = v.to(t.dtype).view_as(t)
    return out


@pytest.mark.parametrize("n", (2, 4))
def test_matches_reference_network(n):
    from splendor.nnet import FoldedNet, SplendorNNet
    with np.load(os.path.join(GOLD, f"nnet_{n}p.npz")) as z:
        g = {k: z[k] for k in z.files}
    net = SplendorNNet(n)
    assert sorted(net.state_dict()) == list(g["keys"])
    assert sum(p.numel() for p in net.parameters()) == int(g["n_params"])
    net.load_state_dict(deterministic_weights(net.state_dict()))
    net.eval()
    b = torch.from_numpy(g["boards"].astype(np.float32))
    valid = torch.from_numpy(g["valid"])
    with torch.no_grad():
        lp, v, sd = net(b, valid)
    m = g["valid"]
    np.testing.assert_allclose(lp.numpy()[m], g["log_pi"][m], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(v.numpy(), g["v"], atol=1e-5)
    np.testing.assert_allclose(sd.numpy(), g["sdiff"], atol=1e-5)
    fold = FoldedNet(net)
    with torch.no_grad():
        pi, v2 = fold(b, valid)
    np.testing.assert_allclose(pi.numpy(), np.exp(g["log_pi"]) * m, atol=1e-6, rtol=1e-4)
    np.testing.assert_allclose(v2.numpy(), g["v"], atol=1e-5)
