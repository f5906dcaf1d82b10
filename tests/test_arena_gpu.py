"""Batched Arena gate against a sequential restatement of Arena.playGames
(Arena.py:66-227) built from the oracle's rules and sequential MCTS: per game two trees
(one per player, persistent within the game), temp-0 move choice with the same Philox
tie-break draw, chance steps on the same Philox stream. Bit-exact move-for-move results."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import _oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

ST_BEST = 6 << 24
DEAL_DRAWS = 29


def oracle_arena(n, G, sims, cpuct, fpu, seed):
    from splendor.arena import one_vs_two
    out = []
    for gid in range(G):
        st, _ = O.init(n, [O.uniform(seed, gid, 0xFFFFFFFF, k) for k in range(DEAL_DRAWS)])
        first = one_vs_two(gid)
        seats = [0] + [1] * (n - 1) if first else [1] + [0] * (n - 1)
        trees = [O.Mcts(n, sims, cpuct, fpu, False) for _ in range(2)]
        result, plies, actions = np.zeros(n, np.float32), 0, []
        for ply in range(62 * n * 2 + 8):
            cur = ply % n
            canon = O.swap_players(n, st, cur) if cur else st.copy()
            k = seats[cur]
            counts = trees[k].search(canon)[0]
            u = O.uniform(seed ^ (k + 1), gid, ST_BEST | ply, 0)
            top = counts.max()
            if top == 0:
                a = int(u * 409)
            else:
                best = np.flatnonzero(counts == top)
                a = int(best[int(u * len(best))])
            assert O.valid_moves(n, canon, 0)[a]
            actions.append(a)
            st, _, _ = O.make_move(n, st, a, cur, False, [O.uniform(seed, gid, ply, d) for d in range(8)])
            r = O.check_end(n, st)
            if r.any():
                result, plies = r, ply + 1
                break
        out.append((result, plies, [O.score(n, st, p) for p in range(n)], actions))
    return out


@pytest.mark.parametrize("n,G,sims", [(2, 12, 6), (4, 6, 4)])
def test_arena_matches_oracle(n, G, sims):
    from splendor.SplendorGame import SplendorGame
    from splendor.arena import BatchedArena, one_vs_two
    from splendor.mcts import HashEvaluator
    seed, cpuct, fpu = 21, 1.5, 0.1
    g = SplendorGame(n)
    args = dict(numMCTSSims=sims, cpuct=cpuct, fpu=fpu, arenaCompare=G)
    ar = BatchedArena(g, None, None, args, batch=G, seed=seed,
               evaluators=(HashEvaluator(g.engine), HashEvaluator(g.engine)))
    one, two, draws = ar.playGames(G)
    ref = oracle_arena(n, G, sims, cpuct, fpu, seed)
    last = ar.last
    for i, (r, plies, score, _) in enumerate(ref):
        np.testing.assert_array_equal(last["result"][i], r, err_msg=f"game {i}")
        assert last["plies"][i] == plies, f"game {i}"
        np.testing.assert_array_equal(last["score"][i], score)
    r0 = np.array([r[0][0] for r in ref])
    ovt = np.array([one_vs_two(i) for i in range(G)])
    assert one == int(np.sum(np.where(ovt, r0 == 1.0, r0 == -1.0)))
    assert two == int(np.sum(np.where(ovt, r0 == -1.0, r0 == 1.0)))
    assert one + two + draws == G
    assert ar.capacity == {"prunes": 0, "resets": 0, "unexpanded": 0}


class NegatedHash:
    """The reference fixture's second network: the hash network with values negated."""

    def __init__(self, engine):
        from splendor.mcts import HashEvaluator
        self.h = HashEvaluator(engine)

    def __call__(self, leaf_state, leaf_mask, leaf_valid):
        pi, v = self.h(leaf_state, leaf_mask, leaf_valid)
        return pi, -v


@pytest.mark.parametrize("n", (2, 3))
def test_arena_matches_reference(n):
    """BatchedArena against Arena.playGames itself (tests/golden/arena_*.npz: the reference
    run with two MCTS players over different hash networks and the build's keyed draws
    injected): every move of every game, per-game results and the totals."""
    import os
    from splendor.SplendorGame import SplendorGame
    from splendor.arena import BatchedArena
    from splendor.mcts import HashEvaluator
    with np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"arena_{n}p.npz")) as z:
        d = {k: z[k] for k in z.files}
    G = len(d["plies"])
    g = SplendorGame(n)
    args = dict(numMCTSSims=int(d["sims"]), cpuct=float(d["cpuct"]), fpu=float(d["fpu"]), arenaCompare=G)
    ar = BatchedArena(g, None, None, args, batch=G, seed=int(d["seed"]),
                      evaluators=(HashEvaluator(g.engine), NegatedHash(g.engine)))
    one, two, draws = ar.playGames(G)
    last = ar.last
    for i in range(G):
        p = int(d["plies"][i])
        assert last["plies"][i] == p, f"game {i}"
        np.testing.assert_array_equal(last["actions"][i][:p], d["actions"][i][:p], err_msg=f"game {i}")
        assert [float(last["result"][i][0]), float(last["score"][i][0]), float(last["score"][i][1])] == \
            list(d["result"][i])
    assert (one, two, draws) == (int(d["one"]), int(d["two"]), int(d["draws"]))


def test_arena_batches_and_gate():
    """Games split over several batches give the same per-game records as one batch with
    the same game ids; the Coach.learn acceptance rule."""
    from splendor.SplendorGame import SplendorGame
    from splendor.arena import BatchedArena, accept_new_network
    from splendor.mcts import HashEvaluator
    g = SplendorGame(2)
    args = dict(numMCTSSims=4, cpuct=1.0, fpu=0.0)
    ev = (HashEvaluator(g.engine), HashEvaluator(g.engine))
    a = BatchedArena(g, None, None, args, batch=8, seed=5, evaluators=ev)
    a.playGames(8)
    b = BatchedArena(g, None, None, args, batch=3, seed=5, evaluators=ev)
    b.playGames(8)
    for k in ("result", "plies", "score", "one_vs_two", "game"):
        np.testing.assert_array_equal(a.last[k], b.last[k], err_msg=k)
    assert accept_new_network(6, 4, 0.55) and not accept_new_network(5, 5, 0.55)
    assert not accept_new_network(0, 0, 0.55)


def test_reference_arena_with_player_callables():
    """Arena(player1, player2, None, game, args).playGames with plain callables (the pit.py
    form): first-legal vs last-legal players; every game ends, counts add up, and game i is
    the same game as a direct Game-API loop with the seats of Arena.py:200-203."""
    from splendor.SplendorGame import SplendorGame
    from splendor.arena import Arena, one_vs_two
    g = SplendorGame(2)
    first = lambda b: int(np.flatnonzero(g.getValidMoves(b, 0))[0])      # noqa: E731
    last = lambda b: int(np.flatnonzero(g.getValidMoves(b, 0))[-1])      # noqa: E731
    ar = Arena(first, last, None, g, None)
    results = [ar.playGame(other_way=not one_vs_two(i))[0] for i in range(4)]
    one, two, draws = Arena(first, last, None, g, None).playGames(4)
    assert one + two + draws == 4
    exp_one = sum(1 for i, r in enumerate(results) if r == (1. if one_vs_two(i) else -1.))
    assert one == exp_one
