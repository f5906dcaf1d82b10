"""Pin the CPU oracle against golden vectors recorded from the reference
(tests/golden/make_golden.py). Everything here is bit-exact."""
import os

import numpy as np
import pytest

import _oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NS = (2, 3, 4)


def load(name):
    with np.load(os.path.join(GOLD, name)) as z:
        return {k: z[k] for k in z.files}


def test_tables_match_reference():
    t = load("tables.npz")
    for tier, key in enumerate(("cards1", "cards2", "cards3")):
        ref = t[key]
        for color in range(5):
            for k in range(ref.shape[1]):
                np.testing.assert_array_equal(O.card(tier, color, k), ref[color, k])


@pytest.mark.parametrize("n", NS)
def test_init_game(n):
    d = load(f"env_{n}p.npz")
    for u, st in zip(d["init_uniforms"], d["init_state"]):
        got, used = O.init(n, u)
        assert used == len(u)
        np.testing.assert_array_equal(got, st)


@pytest.mark.parametrize("n", NS)
def test_valid_moves(n):
    d = load(f"env_{n}p.npz")
    for i in range(len(d["state"])):
        np.testing.assert_array_equal(O.valid_moves(n, d["canon"][i], 0), d["mask_canon"][i], err_msg=f"canon {i}")
        np.testing.assert_array_equal(O.valid_moves(n, d["state"][i], int(d["player"][i])),
                                      d["mask_player"][i], err_msg=f"player view {i}")


@pytest.mark.parametrize("n", NS)
def test_canonical_and_scores(n):
    d = load(f"env_{n}p.npz")
    for i in range(len(d["state"])):
        p = int(d["player"][i])
        got = O.swap_players(n, d["state"][i], p) if p else d["state"][i]
        np.testing.assert_array_equal(got, d["canon"][i])
        assert [O.score(n, d["state"][i], q) for q in range(n)] == list(d["scores"][i])
        np.testing.assert_array_equal(O.check_end(n, d["state"][i]), d["ended"][i])


@pytest.mark.parametrize("n", NS)
def test_chance_steps(n):
    d = load(f"env_{n}p.npz")
    uni = d["uniforms"]
    for i in range(len(d["state"])):
        off, ln = int(d["u_off"][i]), int(d["u_len"][i])
        got, nxt, used = O.make_move(n, d["state"][i], int(d["action"][i]), int(d["player"][i]), False,
                                     uni[off:off + ln])
        assert used == ln, i
        assert nxt == d["next_player"][i]
        np.testing.assert_array_equal(got, d["next_state"][i], err_msg=f"step {i} a={d['action'][i]}")
        np.testing.assert_array_equal(O.check_end(n, got), d["next_ended"][i])


@pytest.mark.parametrize("n", NS)
def test_deterministic_tree_steps(n):
    d = load(f"env_{n}p.npz")
    for j in range(len(d["det_src"])):
        src = d["canon"][int(d["det_src"][j])]
        got, nxt = O.tree_step(n, src, int(d["det_action"][j]))
        assert nxt == d["det_next_player"][j]
        np.testing.assert_array_equal(got, d["det_next_state"][j], err_msg=f"det {j} a={d['det_action'][j]}")


@pytest.mark.parametrize("n", NS)
def test_end_known_answers(n):
    d = load(f"end_{n}p.npz")
    for st, e in zip(d["state"], d["ended"]):
        np.testing.assert_array_equal(O.check_end(n, st), e)


@pytest.mark.parametrize("n", NS)
def test_fake_network(n):
    d = load(f"fakenn_{n}p.npz")
    for st, m, pi, v in zip(d["state"], d["mask"], d["pi"], d["v"]):
        gp, gv = O.fake_predict(n, st, m)
        np.testing.assert_array_equal(gp, pi)
        np.testing.assert_array_equal(gv, v)


def test_numpy_pairwise_sum():
    rng = np.random.default_rng(5)
    for _ in range(300):
        x = (rng.random(409) ** 3).astype(np.float32)
        x[rng.random(409) < 0.9] = 0
        assert O.np_sum_f32(x) == np.sum(x)


@pytest.mark.parametrize("n", (2, 4))
def test_mcts_single_searches(n):
    d = load(f"mcts_{n}p.npz")
    for i in range(len(d["root"])):
        m = O.Mcts(n, int(d["sims"][i]), float(d["cpuct"][i]), float(d["fpu"][i]), bool(d["forced"][i]))
        counts, qsa, probs, q, _ = m.search(d["root"][i])
        np.testing.assert_array_equal(counts, d["counts"][i], err_msg=f"search {i}")
        np.testing.assert_array_equal(qsa, d["qsa"][i])
        np.testing.assert_array_equal(probs, d["probs"][i])
        np.testing.assert_array_equal(q, d["q"][i])


@pytest.mark.parametrize("n", (2, 4))
def test_mcts_multi_move_tree_reuse(n):
    d = load(f"mcts_{n}p.npz")
    m = O.Mcts(n, 50, 2.5, 0.3, False)
    st, used = O.init(n, d["seq_init_uniforms"])
    np.testing.assert_array_equal(st, d["seq_init_state"])
    uni = d["seq_uniforms"]
    player = 0
    for k in range(len(d["seq_root"])):
        canon = O.swap_players(n, st, player) if player else st
        np.testing.assert_array_equal(canon, d["seq_root"][k])
        counts, qsa, probs, q, _ = m.search(canon)
        np.testing.assert_array_equal(counts, d["seq_counts"][k], err_msg=f"move {k}")
        np.testing.assert_array_equal(probs, d["seq_probs"][k])
        np.testing.assert_array_equal(q, d["seq_q"][k])
        a = int(np.argmax(counts))
        assert a == d["seq_action"][k]
        off, ln = int(d["seq_uoff"][k]), int(d["seq_ulen"][k])
        st, player, _ = O.make_move(n, st, a, player, False, uni[off:off + ln])


@pytest.mark.parametrize("n", (2, 4))
def test_mcts_large_budget_searches(n):
    """Round 6: the reference's MCTS executed at BASELINE configs 4 / 5's budgets (2p 1,600, 4p
    400 simulations; genbu.pt's cpuct 2.5 / fpu 0.3) from 10 roots spread over random games,
    6 under the hash network (mode 0) and 4 under the peaked one (mode 1: deep trees). Beyond
    the root statistics, the table size and every simulation's leaf depth (sum, max, count)."""
    d = load(f"bigmcts_{n}p.npz")
    sims = int(d["sims"])
    try:
        for i in range(len(d["root"])):
            O.set_fake_mode(int(d["mode"][i]))
            O.depth_stats(reset=True)
            m = O.Mcts(n, sims, float(d["cpuct"]), float(d["fpu"]), False)
            counts, qsa, probs, q, nodes = m.search(d["root"][i])
            msg = f"root {i} (mode {int(d['mode'][i])})"
            np.testing.assert_array_equal(counts, d["counts"][i], err_msg=msg)
            np.testing.assert_array_equal(qsa, d["qsa"][i], err_msg=msg)
            np.testing.assert_array_equal(probs, d["probs"][i], err_msg=msg)
            np.testing.assert_array_equal(q, d["q"][i], err_msg=msg)
            assert nodes == d["nodes"][i], msg
            assert O.depth_stats(reset=True) == tuple(int(x) for x in d["depth"][i]), msg
    finally:
        O.set_fake_mode(0)
    # the set reaches the deep regime the large-budget self-play tests run in
    deep = d["depth"][d["mode"] == 1]
    assert (deep[:, 1] >= 20).any()


@pytest.mark.parametrize("n", (2, 4))
def test_mcts_large_budget_tree_reuse(n):
    """A 12-move game at the large budget with the tree kept between moves (MCTS.py:79-85
    cleaning included), chance injected, arg-max play."""
    d = load(f"bigmcts_{n}p.npz")
    m = O.Mcts(n, int(d["sims"]), float(d["cpuct"]), float(d["fpu"]), False)
    st, used = O.init(n, d["seq_init_uniforms"])
    np.testing.assert_array_equal(st, d["seq_init_state"])
    uni = d["seq_uniforms"]
    player = 0
    for k in range(len(d["seq_root"])):
        canon = O.swap_players(n, st, player) if player else st
        np.testing.assert_array_equal(canon, d["seq_root"][k])
        counts, qsa, probs, q, _ = m.search(canon)
        np.testing.assert_array_equal(counts, d["seq_counts"][k], err_msg=f"move {k}")
        np.testing.assert_array_equal(probs, d["seq_probs"][k])
        np.testing.assert_array_equal(q, d["seq_q"][k])
        a = int(np.argmax(counts))
        assert a == d["seq_action"][k]
        off, ln = int(d["seq_uoff"][k]), int(d["seq_ulen"][k])
        st, player, _ = O.make_move(n, st, a, player, False, uni[off:off + ln])


def test_philox_known_answer():
    # Random123 Philox4x32-10 known-answer vector (ctr=0,key=0)
    import ctypes as C
    L = O.lib()
    out = (C.c_uint32 * 4)()
    L.or_philox4x32(0, 0, (C.c_uint32 * 4)(0, 0, 0, 0), out)
    assert list(out) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    L.or_philox4x32(0xA4093822, 0x299F31D0,
                    (C.c_uint32 * 4)(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), out)
    assert list(out) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]
    us = [O.uniform(123, b, s, k) for b in range(4) for s in range(4) for k in range(4)]
    assert all(0.0 <= u < 1.0 for u in us) and len(set(us)) == len(us)
    # uniform d = half d&1 of counter block d>>1 (53 bits from two words)
    for d in range(6):
        L.or_philox4x32(7, 0, (C.c_uint32 * 4)(d >> 1, 3, 5, 0x53504C44), out)
        w = list(out)[2 * (d & 1):2 * (d & 1) + 2]
        assert O.uniform(7, 3, 5, d) == ((w[0] >> 5) * 67108864.0 + (w[1] >> 6)) / 9007199254740992.0


def test_symmetries_shapes():
    d = load("env_2p.npz")
    st = d["canon"][40]
    pi = np.random.default_rng(0).random(409).astype(np.float32)
    s, p, v = O.symmetries(2, st, pi, d["mask_canon"][40])
    assert len(s) >= 10
    np.testing.assert_array_equal(s[0], st)
