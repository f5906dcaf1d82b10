"""GPU parity of the device-resident batched MCTS against the reference's MCTS (golden
searches recorded by make_golden.py) and the sequential C oracle. Deterministic hash
network on both sides; Dirichlet off. Bit-exact: visit counts, Q (float64), probs, q."""
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


@pytest.fixture(scope="module")
def engines():
    from splendor.env import SplendorEngine
    return {n: SplendorEngine(n) for n in (2, 3, 4)}


def mcts_for(engine, B, sims, cpuct, fpu, forced, **kw):
    from splendor.mcts import BatchedMCTS
    args = dict(numMCTSSims=sims, cpuct=cpuct, fpu=fpu, prob_fullMCTS=1.0, ratio_fullMCTS=5,
                forced_playouts=forced, dirichletAlpha=0.0, temperature=[1.25, 0.8], tempThreshold=10)
    return BatchedMCTS(engine, B, args, **kw)


@pytest.mark.parametrize("n", (2, 4))
def test_single_searches_match_reference(engines, n):
    d = load(f"mcts_{n}p.npz")
    cases = sorted(set(int(c) for c in d["case"]))
    for c in cases:
        idx = np.flatnonzero(d["case"] == c)
        i0 = idx[0]
        m = mcts_for(engines[n], len(idx), int(d["sims"][i0]), float(d["cpuct"][i0]), float(d["fpu"][i0]),
                     bool(d["forced"][i0]))
        roots = torch.from_numpy(d["root"][idx]).cuda()
        probs, q, full, counts = m.get_action_prob(roots, force_full_search=True, keep_tree=False)
        _, qsa, _, _ = m.root_stats()
        np.testing.assert_array_equal(counts.cpu().numpy(), d["counts"][idx], err_msg=f"case {c}")
        np.testing.assert_array_equal(qsa.cpu().numpy(), d["qsa"][idx])
        np.testing.assert_array_equal(probs.cpu().numpy(), d["probs"][idx])
        np.testing.assert_array_equal(q.cpu().numpy(), d["q"][idx])


@pytest.mark.parametrize("n", (2, 4))
def test_multi_move_tree_reuse_matches_reference(engines, n):
    d = load(f"mcts_{n}p.npz")
    m = mcts_for(engines[n], 1, 50, 2.5, 0.3, False)
    for k in range(len(d["seq_root"])):
        root = torch.from_numpy(d["seq_root"][k][None]).cuda()
        probs, q, _, counts = m.get_action_prob(root, force_full_search=True, keep_tree=True)
        np.testing.assert_array_equal(counts.cpu().numpy()[0], d["seq_counts"][k], err_msg=f"move {k}")
        np.testing.assert_array_equal(probs.cpu().numpy()[0], d["seq_probs"][k])
        np.testing.assert_array_equal(q.cpu().numpy()[0], d["seq_q"][k])


@pytest.mark.parametrize("n", (2, 4))
def test_large_budget_searches_match_reference(engines, n):
    """Round 6: the device's root statistics against the reference's MCTS executed at configs
    4 / 5's budgets (2p 1,600, 4p 400 simulations; `bigmcts_*.npz`), under the hash network and
    under the peaked one (deep trees: leaf depths to ~100), with every simulation's leaf depth
    (sum and maximum per tree) as the reference's recursion reached it."""
    from splendor.mcts import HashEvaluator
    d = load(f"bigmcts_{n}p.npz")
    for mode in (0, 1):
        idx = np.flatnonzero(d["mode"] == mode)
        m = mcts_for(engines[n], len(idx), int(d["sims"]), float(d["cpuct"]), float(d["fpu"]), False,
                     evaluator=HashEvaluator(engines[n], mode=mode))
        probs, q, _, counts = m.get_action_prob(torch.from_numpy(d["root"][idx]).cuda(), force_full_search=True,
                                                keep_tree=False)
        _, qsa, _, _ = m.root_stats()
        msg = f"{n}p mode {mode}"
        np.testing.assert_array_equal(counts.cpu().numpy(), d["counts"][idx], err_msg=msg)
        np.testing.assert_array_equal(qsa.cpu().numpy(), d["qsa"][idx], err_msg=msg)
        np.testing.assert_array_equal(probs.cpu().numpy(), d["probs"][idx], err_msg=msg)
        np.testing.assert_array_equal(q.cpu().numpy(), d["q"][idx], err_msg=msg)
        h = m.headers()
        np.testing.assert_array_equal(h["depth_sum"], d["depth"][idx, 0], err_msg=msg)
        np.testing.assert_array_equal(h["depth_max"], d["depth"][idx, 1], err_msg=msg)
        assert h["prunes"].sum() == h["resets"].sum() == h["unexpanded"].sum() == 0


@pytest.mark.parametrize("n", (2, 4))
def test_large_budget_tree_reuse_matches_reference(engines, n):
    """The reference's 12-move game at the large budget with its tree kept between moves."""
    d = load(f"bigmcts_{n}p.npz")
    m = mcts_for(engines[n], 1, int(d["sims"]), float(d["cpuct"]), float(d["fpu"]), False)
    for k in range(len(d["seq_root"])):
        root = torch.from_numpy(d["seq_root"][k][None]).cuda()
        probs, q, _, counts = m.get_action_prob(root, force_full_search=True, keep_tree=True)
        np.testing.assert_array_equal(counts.cpu().numpy()[0], d["seq_counts"][k], err_msg=f"{n}p move {k}")
        np.testing.assert_array_equal(probs.cpu().numpy()[0], d["seq_probs"][k])
        np.testing.assert_array_equal(q.cpu().numpy()[0], d["seq_q"][k])


@pytest.mark.parametrize("n,sims", [(2, 100), (3, 40), (4, 64)])
def test_batch_searches_match_oracle(engines, n, sims):
    d = load(f"env_{n}p.npz")
    roots = d["canon"][::2][:192]
    m = mcts_for(engines[n], len(roots), sims, 2.5, 0.3, True)
    probs, q, _, counts = m.get_action_prob(torch.from_numpy(roots).cuda(), keep_tree=False)
    counts, probs, q = counts.cpu().numpy(), probs.cpu().numpy(), q.cpu().numpy()
    for b in range(0, len(roots), 7):
        om = O.Mcts(n, sims, 2.5, 0.3, True)
        oc, _, op, oq, _ = om.search(roots[b])
        np.testing.assert_array_equal(counts[b], oc, err_msg=f"root {b}")
        np.testing.assert_array_equal(probs[b], op)
        np.testing.assert_array_equal(q[b], oq)


@pytest.mark.parametrize("boards", (True, False))
def test_persistent_trees_with_gc_match_oracle(engines, boards):
    """64 games x 12 moves: argmax play, chance via Philox, persistent trees + exact GC
    (node boards move with their nodes)."""
    n, B, sims, seed = 2, 64, 60, 77
    e = engines[n]
    m = mcts_for(e, B, sims, 1.5, 0.2, False, node_cap=1024, edge_cap=24576, node_boards=boards)
    st = e.new_state(B)
    player = torch.zeros(B, dtype=torch.int8, device="cuda")
    e.init(st, player, seed=seed, stream=0xFFFFFFFF)
    oracles = [O.Mcts(n, sims, 1.5, 0.2, False) for _ in range(B)]
    host = st.cpu().numpy().copy()
    hp = np.zeros(B, np.int64)
    for mv in range(12):
        canon = e.canonical(st, player)
        probs, q, _, counts = m.get_action_prob(canon, force_full_search=True, keep_tree=True)
        counts = counts.cpu().numpy()
        hdr = m.headers()
        assert hdr["overflow"].max() == 0
        action = counts.argmax(1)
        for b in range(B):
            c = host[b] if hp[b] == 0 else O.swap_players(n, host[b], int(hp[b]))
            oc, _, _, _, _ = oracles[b].search(c)
            np.testing.assert_array_equal(counts[b], oc, err_msg=f"move {mv} game {b}")
            u = [O.uniform(seed, b, 1000 + mv, k) for k in range(2)]
            host[b], hp[b], _ = O.make_move(n, host[b], int(action[b]), int(hp[b]), False, u)
        nxt = torch.empty(B, dtype=torch.int8, device="cuda")
        e.step(st, torch.from_numpy(action.astype(np.int16)).cuda(), player, nxt, deterministic=False,
               seed=seed, stream=1000 + mv)
        player = nxt
        np.testing.assert_array_equal(st.cpu().numpy(), host)
    # the reachable table always fit: no search started on a pruned or emptied tree
    assert hdr["prunes"].sum() == hdr["resets"].sum() == hdr["unexpanded"].sum() == 0
    assert hdr["node_count"].max() <= 1024
