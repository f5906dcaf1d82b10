"""Episode-end example pipeline and the 406 -> 409 policy-head remap
(§8f row 2). CPU only: the columnar ExampleSet against the reference's tuple records
(Coach.py:91-98, GenericNNetWrapper.pick_examples / compute_surprise_weights :326-340)."""
import numpy as np
import pytest
import torch

from splendor.env import ACTIONS, pack_mask, unpack_mask
from splendor.examples import ExampleHistory, ExampleSet
from splendor.nnet import SplendorNNet, remap_policy_head


def _tuples(E, n=2, seed=0):
    rng = np.random.default_rng(seed)
    R = 32 + 10 * n + n * n
    out = []
    for _ in range(E):
        board = rng.integers(-128, 128, size=(R, 7), dtype=np.int8)
        valids = rng.random(ACTIONS) < 0.1
        valids[rng.integers(ACTIONS)] = True
        pi = np.where(valids, rng.random(ACTIONS), 0).astype(np.float32)
        pi /= pi.sum()
        winner = rng.choice([-1.0, 1.0, 0.01], size=n).astype(np.float32)
        scdiff = rng.integers(-15, 16, size=n).astype(np.int32)
        surprise = rng.random(n).astype(np.float32)
        out.append((board, pi, winner, scdiff, valids, surprise))
    return out


def _eq_tuples(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(np.asarray(u), np.asarray(v))


def test_pack_mask_roundtrip():
    v = torch.rand(33, ACTIONS) < 0.3
    v[:, 408] = True
    w = pack_mask(v)
    assert w.shape == (33, 7) and w.dtype == torch.int64
    assert torch.equal(unpack_mask(w), v)


def test_tuples_roundtrip():
    ex = _tuples(50)
    s = ExampleSet.from_tuples(ex)
    assert len(s) == 50
    _eq_tuples(s.to_tuples(), ex)


@pytest.mark.parametrize("compress", [True, False])
def test_save_load(tmp_path, compress):
    ex = _tuples(40, n=4, seed=3)
    s = ExampleSet.from_tuples(ex)
    p = str(tmp_path / "it1.npz")
    s.save(p, compress=compress)
    t = ExampleSet.load(p)
    _eq_tuples(t.to_tuples(), ex)


def test_pick_examples_matches_reference_layout():
    ex = _tuples(64, seed=5)
    s = ExampleSet.from_tuples(ex)
    ids = np.random.default_rng(1).choice(64, size=16, replace=False)
    ref = list(zip(*[ex[i] for i in ids]))              # GenericNNetWrapper.pick_examples
    got = s.pick_examples(ids)
    assert len(got) == len(ref) == 6
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g.numpy(), np.stack(r))


def test_surprise_weights_match_reference_formula():
    ex = _tuples(30, seed=7)
    s = ExampleSet.from_tuples(ex)
    sur = np.array([x[-1] for x in ex])                  # GenericNNetWrapper.py:335-339
    w = sur / sur.sum() + 1. / len(sur)
    w = w / w.sum()
    np.testing.assert_allclose(s.compute_surprise_weights(), w, rtol=1e-12)


def test_history_window_and_file(tmp_path):
    h = ExampleHistory(max_iters=2)
    sets = [_tuples(k, seed=k) for k in (5, 7, 9)]
    for t in sets:
        h.append(ExampleSet.from_tuples(t))
    assert len(h.iters) == 2 and len(h) == 16            # oldest iteration dropped
    h.save(str(tmp_path))
    g = ExampleHistory.load(str(tmp_path), max_iters=2)
    assert [len(x) for x in g.iters] == [7, 9]
    _eq_tuples(g.iters[0].to_tuples(), sets[1])
    _eq_tuples(g.merged().to_tuples(), sets[1] + sets[2])


def test_example_file_has_no_pickles(tmp_path):
    s = ExampleSet.from_tuples(_tuples(3))
    p = str(tmp_path / "x.npz")
    s.save(p)
    with np.load(p, allow_pickle=False) as z:            # would raise on object arrays
        assert all(z[k].dtype != object for k in z.files)


def test_remap_406_policy_head():
    torch.manual_seed(0)
    old = SplendorNNet(2, action_size=406).eval()
    for m in old.modules():                              # non-trivial BN statistics
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.uniform_(-0.5, 0.5)
            m.running_var.uniform_(0.5, 2.0)
    new = SplendorNNet(2).eval()
    new.load_state_dict(remap_policy_head(old.state_dict()))
    g = torch.Generator().manual_seed(1)
    board = torch.randint(-3, 8, (16, 56, 7), generator=g).float()
    v406 = torch.rand(16, 406, generator=g) < 0.2
    v406[:, 405] |= torch.rand(16, generator=g) < 0.5    # pass sometimes legal
    v406[:, 0] = True
    v409 = torch.zeros(16, ACTIONS, dtype=torch.bool)
    v409[:, :405] = v406[:, :405]
    v409[:, 408] = v406[:, 405]
    with torch.no_grad():
        lp_o, v_o, _ = old(board, v406)
        lp_n, v_n, _ = new(board, v409)
    torch.testing.assert_close(v_n, v_o, rtol=0, atol=0)
    p_o, p_n = lp_o.exp(), lp_n.exp()
    torch.testing.assert_close(p_n[:, :405], p_o[:, :405], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(p_n[:, 408], p_o[:, 405], rtol=1e-6, atol=1e-7)
    assert float(p_n[:, 405:408].abs().max()) == 0.0


def test_remap_rejects_other_sizes():
    sd = SplendorNNet(2, action_size=300).state_dict()
    with pytest.raises(ValueError):
        remap_policy_head(sd)
    same = SplendorNNet(2).state_dict()
    assert remap_policy_head(same)["output_layers_PI.1.weight"] is same["output_layers_PI.1.weight"]
