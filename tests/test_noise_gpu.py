"""GPU parity of root Dirichlet noise (MCTS.py:141-154, 180-186, 239-250): device searches
with noise on against the reference's searches recorded with the same injected Dirichlet
vectors (tests/golden/noisesearch_*.npz), the stored root priors against the oracle's
noise restatement (pinned by noise_*.npz), including 4-player roots with more than 192
legal actions. Bit-exact."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import _oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLD, name)) as z:
        return {k: z[k] for k in z.files}


def mcts_for(engine, B, sims, cpuct, fpu, forced, alpha, t0, seed, board_base):
    from splendor.mcts import BatchedMCTS
    args = dict(numMCTSSims=sims, cpuct=cpuct, fpu=fpu, prob_fullMCTS=1.0, ratio_fullMCTS=5,
                forced_playouts=forced, dirichletAlpha=alpha, temperature=[t0, 0.8], tempThreshold=10)
    return BatchedMCTS(engine, B, args, dirichlet_noise=True, seed=seed, board_base=board_base)


@pytest.mark.parametrize("n", (2, 3, 4))
def test_noised_searches_match_reference(n):
    """Search 1 noises a new root (raw network priors), search 2 re-noises the stored priors
    of the kept root; counts, Q, probs, q and the stored priors."""
    from splendor.env import SplendorEngine
    e = SplendorEngine(n)
    d = load(f"noisesearch_{n}p.npz")
    seed = 3100 + n
    for c in sorted(set(int(x) for x in d["case"])):
        idx = np.flatnonzero(d["case"] == c)
        i0 = idx[0]
        assert np.array_equal(d["board"][idx], d["board"][i0] + np.arange(len(idx)))
        m = mcts_for(e, len(idx), int(d["sims"][i0]), float(d["cpuct"][i0]), float(d["fpu"][i0]),
                     bool(d["forced"][i0]), float(d["alpha"][i0]), float(d["temp0"][i0]), seed, int(d["board"][i0]))
        roots = torch.from_numpy(d["root"][idx]).cuda()
        for s in (1, 2):
            probs, q, _, counts = m.get_action_prob(roots, force_full_search=True, keep_tree=(s == 2))
            _, qsa, _, _ = m.root_stats()
            np.testing.assert_array_equal(counts.cpu().numpy(), d[f"counts{s}"][idx], err_msg=f"case {c} search {s}")
            np.testing.assert_array_equal(qsa.cpu().numpy(), d[f"qsa{s}"][idx])
            np.testing.assert_array_equal(probs.cpu().numpy(), d[f"probs{s}"][idx])
            np.testing.assert_array_equal(q.cpu().numpy(), d[f"q{s}"][idx])
        ps = m.root_priors().cpu().numpy()
        assert np.allclose(ps.sum(1, dtype=np.float64), 1.0, atol=1e-5)


@pytest.mark.parametrize("n,B,sims", [(4, 64, 12), (2, 64, 12)])
def test_wide_roots_noised_priors_match_oracle(n, B, sims):
    """Roots with every exchange family open (4p: up to 230 legal actions, > 3 x 64 lanes):
    the device's noised priors equal the oracle's softmax -> Dirichlet mix -> normalise, they
    sum to 1, and the searches agree."""
    from splendor.env import SplendorEngine
    from splendor.mcts import HashEvaluator
    e = SplendorEngine(n)
    env = load(f"env_{n}p.npz")
    base = env["canon"][::5][:B].copy()
    total = {2: 4, 3: 5, 4: 7}[n]
    for st in base:                                           # make_golden.wide_roots
        st[32 + n:32 + 2 * n, :6] = 0
        st[32 + n, :5] = 2
        st[0, :5] = total - 2
        st[0, 5] = 5
    legal = np.array([O.valid_moves(n, st, 0).sum() for st in base])
    if n == 4:
        assert legal.max() > 192
    seed, bb, alpha, t0 = 91, 500, 0.3, 1.25
    m = mcts_for(e, B, sims, 1.5, 0.1, False, alpha, t0, seed, bb)
    m.evaluator = HashEvaluator(e)
    probs, q, _, counts = m.get_action_prob(torch.from_numpy(base).cuda(), force_full_search=True, keep_tree=False)
    ps = m.root_priors().cpu().numpy()
    counts = counts.cpu().numpy()
    for t in range(B):
        va = O.valid_moves(n, base[t], 0)
        raw, _ = O.fake_predict(n, base[t], va)
        dirv = O.dirichlet(alpha, seed, bb + t, O.ST_DIR | 1, int(va.sum()))
        want = O.root_noise(raw, va, dirv, t0)
        np.testing.assert_array_equal(ps[t], want, err_msg=f"root {t} ({legal[t]} legal)")
        om = O.Mcts(n, sims, 1.5, 0.1, False)
        om.set_noise(alpha, t0, seed, bb + t, O.ST_DIR | 1)
        np.testing.assert_array_equal(counts[t], om.search(base[t])[0], err_msg=f"root {t}")
    assert np.allclose(ps.sum(1, dtype=np.float64), 1.0, atol=1e-5)
