"""The reference's plug-in surface over the HIP engine: SplendorGame (Game API), MCTS
(getActionProb), NNetWrapper (predict), Coach (executeEpisode), Arena-style play."""
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
def game2():
    from splendor.SplendorGame import SplendorGame
    return SplendorGame(2, seed=11)


def test_game_api_matches_reference(game2):
    g, d = game2, load("env_2p.npz")
    for i in range(0, len(d["state"]), 9):
        st, p = d["state"][i], int(d["player"][i])
        np.testing.assert_array_equal(g.getValidMoves(st, p), d["mask_player"][i].astype(bool))
        np.testing.assert_array_equal(g.getCanonicalForm(st, p), d["canon"][i])
        np.testing.assert_array_equal(g.getGameEnded(st, p), d["ended"][i])
        assert [g.getScore(st, q) for q in range(2)] == list(d["scores"][i])
        assert g.getRound(st) == d["round"][i]
        assert g.stringRepresentation(st) == st.tobytes()
    for j in range(0, len(d["det_src"]), 13):
        src = d["canon"][int(d["det_src"][j])]
        nxt, np_ = g.getNextState(src, 0, int(d["det_action"][j]), deterministic=True)
        if np_ != 0:
            nxt = g.getCanonicalForm(nxt, np_)
        np.testing.assert_array_equal(nxt, d["det_next_state"][j])
    assert g.getBoardSize() == (56, 7) and g.getActionSize() == 409 and g.getMaxScoreDiff() == 15


def test_chance_next_state_matches_oracle(game2):
    g, d = game2, load("env_2p.npz")
    for i in range(0, len(d["state"]), 17):
        st, p, a = d["state"][i], int(d["player"][i]), int(d["action"][i])
        stream = (7 << 24) | ((g._calls + 1) & 0x00FFFFFF)
        got, nxt = g.getNextState(st, p, a)
        u = [O.uniform(g.seed, 0, stream, k) for k in range(2)]
        ref, rn, _ = O.make_move(2, st, a, p, False, u)
        np.testing.assert_array_equal(got, ref)
        assert nxt == rn


@pytest.mark.parametrize("n", (2, 4))
def test_symmetries_match_oracle(n):
    from splendor.SplendorGame import SplendorGame
    g, d = SplendorGame(n), load(f"env_{n}p.npz")
    rng = np.random.default_rng(1)
    for i in range(0, len(d["canon"]), 23):
        st, va = d["canon"][i], d["mask_canon"][i]
        pi = rng.random(409).astype(np.float32)
        got = g.getSymmetries(st, pi, va.astype(bool))
        os_, op, ov = O.symmetries(n, st, pi, va)
        assert len(got) == len(os_)
        for (b, p, v), rb, rp, rv in zip(got, os_, op, ov):
            np.testing.assert_array_equal(b, rb)
            np.testing.assert_array_equal(p, rp)
            np.testing.assert_array_equal(v, rv.astype(bool))


class HashNet:
    """reference-style nnet with .predict(board, valids) = the oracle's hash network"""

    def __init__(self, n):
        self.n = n

    def predict(self, board, valid_actions):
        return O.fake_predict(self.n, board, np.asarray(valid_actions, np.uint8))


def test_mcts_plugin_matches_reference_searches(game2):
    from splendor.search import MCTS
    d = load("mcts_2p.npz")
    for i in range(0, len(d["root"]), 5):
        args = dict(numMCTSSims=int(d["sims"][i]), cpuct=float(d["cpuct"][i]), fpu=float(d["fpu"][i]),
                    prob_fullMCTS=1.0, ratio_fullMCTS=5, forced_playouts=bool(d["forced"][i]),
                    no_mem_optim=False, dirichletAlpha=0.0, temperature=[1.25, 0.8], tempThreshold=10)
        m = MCTS(game2, HashNet(2), args)
        probs, q, full = m.getActionProb(d["root"][i], temp=1, force_full_search=True)
        np.testing.assert_array_equal(np.array(probs), d["probs"][i])
        np.testing.assert_array_equal(np.array(q), d["q"][i])
        assert full


def test_arena_style_game_and_coach(game2):
    """Two MCTS players (SplendorNNet on device) play a game through the Game API
    (Arena.playGame loop, Arena.py:64-173), then Coach produces training examples."""
    from splendor.NNet import NNetWrapper
    from splendor.search import MCTS
    from splendor.coach import Coach
    g = game2
    args = dict(numMCTSSims=16, cpuct=2.5, fpu=0.3, prob_fullMCTS=1.0, ratio_fullMCTS=5,
                forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    nets = [NNetWrapper(g, seed=s) for s in (1, 2)]
    players = [MCTS(g, nets[k], args) for k in range(2)]
    board, cur = g.getInitBoard(), 0
    for _ in range(300):
        canon = g.getCanonicalForm(board, cur)
        probs, _, _ = players[cur].getActionProb(canon, temp=0, force_full_search=True)
        a = int(np.argmax(probs))
        assert g.getValidMoves(canon, 0)[a]
        board, cur = g.getNextState(board, cur, a)
        if g.getGameEnded(board, cur).any():
            break
    assert g.getGameEnded(board, cur).any()
    MCTS.reset_all_search_trees()
    coach = Coach(g, nets[0], dict(args, prob_fullMCTS=0.25, numMCTSSims=8), batch=64)
    ex = coach.executeEpisodes(8)
    assert len(ex) > 0
    b, pi, win, sd, va, sur = ex[0]
    assert b.shape == (56, 7) and pi.shape == (409,) and va.dtype == bool
    assert abs(float(pi.sum()) - 1) < 1e-5 and set(win.tolist()) <= {-1.0, 1.0, np.float32(0.01)}
