"""Pin the oracle's root noise, symmetries, self-play episode and arena pieces against the
reference (tests/golden/{noise,noisesearch,sym,episode,arena}_*.npz, recorded by
make_golden.py from the reference source with the build's keyed random draws injected).
Everything here is bit-exact."""
import os
import sys

import numpy as np
import pytest

import _oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
import detrand  # noqa: E402


def load(name):
    with np.load(os.path.join(GOLD, name)) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("n", (2, 3, 4))
def test_dirichlet_sampler_matches_restatement(n):
    """or_dirichlet (C) == detrand.dirichlet (Python), the vectors injected into the reference."""
    d = load(f"noise_{n}p.npz")
    for i in range(len(d["ps_in"])):
        k = int(d["vs"][i].sum())
        seed, board, stream = (int(x) for x in d["key"][i])
        got = O.dirichlet(float(d["alpha"][i]), seed, board, stream, k)
        np.testing.assert_array_equal(got, d["dir"][i][:k], err_msg=f"case {i}")


def test_dirichlet_sampler_statistics():
    """The sampler is a Dirichlet(alpha): component means 1/k, variances
    (1/k)(1-1/k)/(k alpha + 1)."""
    alpha, k, reps = 0.3, 20, 400
    x = np.array([O.dirichlet(alpha, 11, r, 2 << 24, k) for r in range(reps)])
    assert np.allclose(x.sum(1), 1.0, atol=1e-12)
    m = x.mean(0)
    assert abs(m.mean() - 1 / k) < 1e-12
    var = (1 / k) * (1 - 1 / k) / (k * alpha + 1)
    assert np.all(np.abs(m - 1 / k) < 5 * np.sqrt(var / reps))
    assert 0.7 < x.var(0).mean() / var < 1.3
    # transcendental helpers vs the Python restatement on awkward arguments
    for v in (1e-300, 2.2e-308 * 4, 0.5, 1.0, 1.4142135623730951, 3.0, 1e300):
        assert detrand.det_log(v) == pytest.approx(np.log(v), rel=1e-15, abs=1e-300)


@pytest.mark.parametrize("n", (2, 3, 4))
def test_root_noise_matches_reference(n):
    """softmax(Ps, T0) -> applyDirNoise -> normalise (MCTS.py:141-144, :150-154), incl.
    roots with more than 192 legal actions (4p)."""
    d = load(f"noise_{n}p.npz")
    if n == 4:
        assert d["vs"].sum(1).max() > 192
    for i in range(len(d["ps_in"])):
        k = int(d["vs"][i].sum())
        got = O.root_noise(d["ps_in"][i], d["vs"][i], d["dir"][i][:k], float(d["temp0"][i]))
        np.testing.assert_array_equal(got, d["ps_out"][i], err_msg=f"case {i}")


@pytest.mark.parametrize("n", (2, 3, 4))
def test_noised_searches_match_reference(n):
    """Full searches with root noise, twice per tree (new root, then re-noised stored priors)."""
    d = load(f"noisesearch_{n}p.npz")
    seed = 3100 + n
    for i in range(len(d["root"])):
        m = O.Mcts(n, int(d["sims"][i]), float(d["cpuct"][i]), float(d["fpu"][i]), bool(d["forced"][i]))
        for s in (1, 2):
            m.set_noise(float(d["alpha"][i]), float(d["temp0"][i]), seed, int(d["board"][i]), O.ST_DIR | s)
            counts, qsa, probs, q, _ = m.search(d["root"][i])
            np.testing.assert_array_equal(counts, d[f"counts{s}"][i], err_msg=f"root {i} search {s}")
            np.testing.assert_array_equal(qsa, d[f"qsa{s}"][i])
            np.testing.assert_array_equal(probs, d[f"probs{s}"][i])
            np.testing.assert_array_equal(q, d[f"q{s}"][i])


@pytest.mark.parametrize("n", (2, 3, 4))
def test_symmetries_match_reference(n):
    """Board.get_symmetries (SplendorLogicNumba.py:349-395) via SplendorGame.getSymmetries."""
    d = load(f"sym_{n}p.npz")
    off = d["off"]
    assert any(off[i + 1] - off[i] > 10 for i in range(len(d["src"])))     # reserve permutations hit
    for i in range(len(d["src"])):
        s, p, v = O.symmetries(n, d["src"][i], d["src_pi"][i], d["src_valids"][i])
        lo, hi = off[i], off[i + 1]
        assert len(s) == hi - lo, f"position {i}"
        np.testing.assert_array_equal(s, d["state"][lo:hi])
        np.testing.assert_array_equal(p, d["pi"][lo:hi])
        np.testing.assert_array_equal(v, d["valids"][lo:hi])


def expand(n, ex, lo, hi):
    """Oracle examples [lo, hi) -> the reference's example list: getSymmetries of each
    recorded position in order, winner / scdiff / surprise shared by the variants."""
    out = {k: [] for k in ("board", "pi", "valids", "winner", "scdiff", "surprise")}
    for j in range(lo, hi):
        va = np.unpackbits(ex["valids"][j].view(np.uint8), bitorder="little")[:409]
        s, p, v = O.symmetries(n, ex["ex_board"][j], ex["pi"][j], va)
        for a, b, c in zip(s, p, v):
            out["board"].append(a)
            out["pi"].append(b)
            out["valids"].append(c)
            out["winner"].append(ex["winner"][j])
            out["scdiff"].append(ex["scdiff"][j])
            out["surprise"].append(ex["surprise"][j])
    return {k: np.array(v) for k, v in out.items()}


@pytest.mark.parametrize("tag", ("2p", "2p_forced", "4p"))
def test_episode_matches_reference(tag):
    """Coach.executeEpisode (Coach.py:50-100) with root noise, temperature sampling, chance,
    examples with symmetries: the oracle's self-play loop (one game per board id) produces
    the reference's example list exactly."""
    d = load(f"episode_{tag}.npz")
    n = {56: 2, 71: 3, 88: 4}[d["board"].shape[1]]
    seed = int(d["seed"])
    a = {k[4:]: d[k] for k in d if k.startswith("arg_")}
    sims, ratio = int(a["numMCTSSims"]), int(a["ratio_fullMCTS"])
    for gi, gb in enumerate(d["game_board_id"]):
        moves = int(d["game_moves"][gi])
        ref = O.selfplay_run(n, 1, moves * sims, seed, sims, ratio, float(a["prob_fullMCTS"]), float(a["cpuct"]),
                             float(a["fpu"]), bool(a["forced_playouts"]), int(a["tempThreshold"]),
                             board_base=int(gb), max_ex=4000, dir_alpha=float(a["dirichletAlpha"]),
                             dir_temp=float(a["temperature"][0]))
        first = np.flatnonzero(ref["meta"][:, 1] == 0)
        assert len(first) and ref["hdr"][0, 4] >= 1, "episode did not finish"
        got = expand(n, ref, first[0], first[-1] + 1)
        sel = d["game"] == gi
        assert len(got["board"]) == int(sel.sum()) == int(d["game_n_examples"][gi])
        np.testing.assert_array_equal(got["board"], d["board"][sel])
        np.testing.assert_array_equal(got["pi"], d["pi"][sel])
        np.testing.assert_array_equal(got["valids"], d["valids"][sel])
        np.testing.assert_array_equal(got["winner"], d["winner"][sel])
        np.testing.assert_array_equal(got["scdiff"], d["scdiff"][sel])
        np.testing.assert_array_equal(got["surprise"], d["surprise"][sel].astype(np.float32))


@pytest.mark.parametrize("n", (2, 3))
def test_arena_matches_reference(n):
    """Arena.playGames (Arena.py:175-227): move-for-move, per-game results and totals."""
    d = load(f"arena_{n}p.npz")
    G = len(d["plies"])
    games = O.arena_play(n, G, int(d["sims"]), float(d["cpuct"]), float(d["fpu"]), int(d["seed"]), neg2=True)
    one = two = 0
    for g, (res, plies, scores, actions) in enumerate(games):
        assert plies == d["plies"][g], f"game {g}"
        np.testing.assert_array_equal(actions, d["actions"][g][:plies])
        assert [res[0], scores[0], scores[1]] == list(d["result"][g])
        ovt = O.one_vs_two(g)
        one += res[0] == (1.0 if ovt else -1.0)
        two += res[0] == (-1.0 if ovt else 1.0)
    assert (one, two, G - one - two) == (int(d["one"]), int(d["two"]), int(d["draws"]))


def test_parallel_oracle_selfplay_equals_serial():
    """The parallel oracle driver (board-id parts in worker processes, used by the GPU
    large-budget parity tests) equals one sequential run, lags included."""
    args = (2, 12, 700, 11, 30, 5, 0.25, 2.5, 0.3, False, 10)
    kw = dict(max_ex=4000, dir_alpha=0.3, dir_temp=1.25, fake_mode=1)
    ref = O.selfplay_run(*args, **kw)
    par = O.selfplay_run_parallel(*args, workers=3, **kw)
    for k in ("hdr", "board", "ex_board", "pi", "valids", "winner", "scdiff", "surprise", "meta"):
        np.testing.assert_array_equal(par[k], ref[k], err_msg=k)
    assert par["depth"] == ref["depth"]
    lag = np.array([0] * 6 + [3] * 6)
    par = O.selfplay_run_parallel(*args, lag=lag, workers=4, **kw)
    a = O.selfplay_run(2, 6, 700, 11, *args[4:], **kw)
    b = O.selfplay_run(2, 6, 697, 11, *args[4:], board_base=6, **kw)
    np.testing.assert_array_equal(par["hdr"], np.concatenate([a["hdr"], b["hdr"]]))
