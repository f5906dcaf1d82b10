"""GPU parity of the HIP env kernels (libsplendor_amd.so via the C ABI) against the CPU
oracle and the reference golden vectors. Bit-exact everywhere (integer/byte work)."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import _oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NS = (2, 3, 4)


def load(name):
    with np.load(os.path.join(GOLD, name)) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def engines():
    from splendor.env import SplendorEngine
    return {n: SplendorEngine(n) for n in NS}


def dev(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def host_mask(words):
    from splendor.env import unpack_mask
    return unpack_mask(words).cpu().numpy().astype(np.uint8)


@pytest.mark.parametrize("n", NS)
def test_valid_moves_matches_reference(engines, n):
    e, d = engines[n], load(f"env_{n}p.npz")
    m = host_mask(e.valid_moves(dev(d["canon"])))
    np.testing.assert_array_equal(m, d["mask_canon"])
    m2 = host_mask(e.valid_moves(dev(d["state"]), dev(d["player"], torch.int8)))
    np.testing.assert_array_equal(m2, d["mask_player"])


@pytest.mark.parametrize("n", NS)
def test_canonical_matches_reference(engines, n):
    e, d = engines[n], load(f"env_{n}p.npz")
    out = e.canonical(dev(d["state"]), dev(d["player"], torch.int8)).cpu().numpy()
    np.testing.assert_array_equal(out, d["canon"])


@pytest.mark.parametrize("n", NS)
def test_game_ended_matches_reference(engines, n):
    e, d, k = engines[n], load(f"env_{n}p.npz"), load(f"end_{n}p.npz")
    np.testing.assert_array_equal(e.game_ended(dev(d["next_state"])).cpu().numpy(), d["next_ended"])
    np.testing.assert_array_equal(e.game_ended(dev(d["state"])).cpu().numpy(), d["ended"])
    np.testing.assert_array_equal(e.game_ended(dev(k["state"])).cpu().numpy(), k["ended"])
    sc = e.score(dev(d["state"])).cpu().numpy()
    np.testing.assert_array_equal(sc, d["scores"])
    np.testing.assert_array_equal(e.round(dev(d["state"])).cpu().numpy(), d["round"])


@pytest.mark.parametrize("n", NS)
def test_chance_step_matches_reference(engines, n):
    e, d = engines[n], load(f"env_{n}p.npz")
    B = len(d["state"])
    u = np.zeros((B, 4), np.float64)
    for i in range(B):
        off, ln = int(d["u_off"][i]), int(d["u_len"][i])
        u[i, :ln] = d["uniforms"][off:off + ln]
    st = dev(d["state"])
    nxt = torch.empty(B, dtype=torch.int8, device="cuda")
    e.step(st, dev(d["action"], torch.int16), dev(d["player"], torch.int8), nxt, deterministic=False,
           uniforms=dev(u))
    np.testing.assert_array_equal(st.cpu().numpy(), d["next_state"])
    np.testing.assert_array_equal(nxt.cpu().numpy(), d["next_player"])


@pytest.mark.parametrize("n", NS)
def test_deck_draw_boundary_uniforms(engines, n):
    """Deck draws with uniforms on (and one ulp around) the cumulative-fraction boundaries
    k / tot and k / nbits, where the device's integer pick defers to the reference's fp
    cumulative sums: every visible-card buy and every deck reserve of the golden states."""
    e, d = engines[n], load(f"env_{n}p.npz")
    base = [j / t for t in range(1, 41) for j in range(t)] + [1 - 2 ** -53]
    cand = np.unique(np.concatenate([base, np.nextafter(base, 0), np.nextafter(base, 1)]))
    cand = cand[(cand >= 0) & (cand < 1)]
    rng = np.random.default_rng(5 + n)
    st0, pl0 = d["state"], d["player"]
    states, players, acts, us = [], [], [], []
    for i in range(len(st0)):
        m = O.valid_moves(n, st0[i], int(pl0[i]))
        for a in np.flatnonzero(m[:27]):             # buys of visible cards and reserves
            for _ in range(3):
                states.append(st0[i]); players.append(pl0[i]); acts.append(a)
                us.append(rng.choice(cand, 2))
    B = len(states)
    st, pl, ac, u = np.stack(states), np.array(players, np.int8), np.array(acts, np.int16), np.stack(us)
    want = np.stack([O.make_move(n, st[b], int(ac[b]), int(pl[b]), False, u[b])[0] for b in range(B)])
    dst = dev(st)
    e.step(dst, dev(ac), dev(pl), None, deterministic=False, uniforms=dev(np.ascontiguousarray(u)))
    np.testing.assert_array_equal(dst.cpu().numpy(), want)


@pytest.mark.parametrize("n", NS)
def test_tree_step_matches_reference(engines, n):
    e, d = engines[n], load(f"env_{n}p.npz")
    parents = d["canon"][d["det_src"]]
    child = e.tree_step(dev(parents), dev(d["det_action"], torch.int16)).cpu().numpy()
    np.testing.assert_array_equal(child, d["det_next_state"])
    # deterministic spl_step + canonical == tree_step
    st = dev(parents)
    nxt = torch.empty(len(parents), dtype=torch.int8, device="cuda")
    e.step(st, dev(d["det_action"], torch.int16), None, nxt, deterministic=True)
    np.testing.assert_array_equal(nxt.cpu().numpy(), d["det_next_player"])
    np.testing.assert_array_equal(e.canonical(st, nxt).cpu().numpy(), d["det_next_state"])


@pytest.mark.parametrize("n", NS)
def test_init_matches_reference(engines, n):
    e, d = engines[n], load(f"env_{n}p.npz")
    G = len(d["init_state"])
    u = np.zeros((G, 32), np.float64)
    u[:, :d["init_uniforms"].shape[1]] = d["init_uniforms"]
    st = e.new_state(G)
    e.init(st, uniforms=dev(u))
    np.testing.assert_array_equal(st.cpu().numpy(), d["init_state"])


@pytest.mark.parametrize("n", NS)
def test_fused_rollout_matches_oracle(engines, n):
    from splendor.env import RolloutBatch
    B, T, seed = 1024, 96, 0x5EED + n
    ref = O.rollout_run(n, B, T, seed)
    rb = RolloutBatch(engines[n], B, seed=seed)
    for t in range(T):
        rb.step()
        np.testing.assert_array_equal(rb.action.cpu().numpy(), ref["action"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(rb.ended.cpu().numpy(), ref["ended"][t])
    np.testing.assert_array_equal(rb.state.cpu().numpy(), ref["state"])
    np.testing.assert_array_equal(rb.player.cpu().numpy(), ref["player"])
    np.testing.assert_array_equal(rb.games.cpu().numpy(), ref["games"])


@pytest.mark.parametrize("n", NS)
def test_rollout_run_matches_oracle(engines, n):
    """spl_rollout_run (K moves per launch, boards kept on chip) == the oracle's move loop,
    across launch boundaries (chunks 1, 40, 55), incl. every move's legality mask."""
    from splendor.env import RolloutBatch
    B, seed = 1000, 0x5EED + 7 * n          # ragged: last workgroup holds 40 boards
    chunks = (1, 40, 55)
    T = sum(chunks)
    ref = O.rollout_run(n, B, T, seed, masks=True)
    rb = RolloutBatch(engines[n], B, seed=seed)
    acts, ends, masks = [], [], []
    for K in chunks:
        o = rb.run(K)
        acts.append(o["action"].cpu().numpy()); ends.append(o["ended"].cpu().numpy())
        masks.append(o["mask"].cpu().numpy().view(np.uint64))
    act, end, msk = np.concatenate(acts), np.concatenate(ends), np.concatenate(masks)
    np.testing.assert_array_equal(act, ref["action"])
    np.testing.assert_array_equal(end, ref["ended"])
    np.testing.assert_array_equal(msk, ref["masks"])      # every word of every move's mask
    np.testing.assert_array_equal(rb.state.cpu().numpy(), ref["state"])
    np.testing.assert_array_equal(rb.player.cpu().numpy(), ref["player"])
    np.testing.assert_array_equal(rb.games.cpu().numpy(), ref["games"])


@pytest.mark.parametrize("n", NS)
def test_long_launch_deal_records_and_fallback(engines, n):
    """One launch of 400 moves: games 1-2 of every board start from the deal records drawn
    at launch start, later games from deals drawn on the spot — both keyed by game number,
    so the result equals the oracle's loop."""
    from splendor.env import RolloutBatch
    B, T, seed = 256, {2: 400, 3: 800, 4: 1200}[n], 0x5EED + 11 * n
    ref = O.rollout_run(n, B, T, seed)
    rb = RolloutBatch(engines[n], B, seed=seed)
    o = rb.run(T)
    assert ref["games"].max() >= 3                    # some boards used the fallback path
    np.testing.assert_array_equal(o["action"].cpu().numpy(), ref["action"])
    np.testing.assert_array_equal(o["ended"].cpu().numpy(), ref["ended"])
    np.testing.assert_array_equal(rb.state.cpu().numpy(), ref["state"])
    np.testing.assert_array_equal(rb.games.cpu().numpy(), ref["games"])


def test_rollout_requires_game_counters(engines):
    from splendor import _lib
    e = engines[2]
    B = 64
    st = e.new_state(B)
    pl = torch.zeros(B, dtype=torch.int8, device="cuda")
    mask = torch.zeros((B, 7), dtype=torch.int64, device="cuda")
    act = torch.zeros(B, dtype=torch.int16, device="cuda")
    end = torch.zeros((B, 2), dtype=torch.float32, device="cuda")
    with pytest.raises(_lib.EngineError):
        e.rollout_step(st, pl, mask, act, end, None, 1, 0)


@pytest.mark.parametrize("n", NS)
def test_rollout_masks_on_perturbed_boards(engines, n):
    """The fused kernel's lane-per-board mask (byte-SAD / lookup fast path and the exact
    path for boards with negative bytes) == the oracle's valid_moves, on golden states whose
    bank / gem / card / cost / deck bytes are randomly overwritten (arbitrary int8)."""
    from splendor.env import MASK_WORDS
    d = load(f"env_{n}p.npz")
    rng = np.random.default_rng(11 + n)
    R = O.rows(n)
    st = np.repeat(d["state"], 3, axis=0)[:600].copy()
    pl = np.repeat(d["player"], 3, axis=0)[:600].astype(np.int8)
    B = len(st)
    rows_hit = np.array([0] + list(range(1, 31)) + list(range(32 + n, R)))
    for b in range(B):
        k = rng.integers(1, 6)
        for _ in range(k):
            r, c = rng.choice(rows_hit), rng.integers(0, 7)
            lo = -128 if b % 3 == 0 else 0           # a third of the boards leave the fast domain
            st[b, r, c] = rng.integers(lo, 12)
    want = np.stack([O.valid_moves(n, st[b], int(pl[b])) for b in range(B)]).astype(np.uint8)
    e = engines[n]
    dst, dpl = dev(st), dev(pl)
    mask = torch.zeros((B, MASK_WORDS), dtype=torch.int64, device="cuda")
    act = torch.zeros(B, dtype=torch.int16, device="cuda")
    end = torch.zeros((B, n), dtype=torch.float32, device="cuda")
    games = torch.zeros(B, dtype=torch.int32, device="cuda")
    e.rollout_step(dst, dpl, mask, act, end, games, 0x5EED, 0)
    np.testing.assert_array_equal(host_mask(mask), want)


def _invariants(n, st, gems_in_play):
    R = 32 + 10 * n + n * n
    gems = 32 + n
    cards = 32 + 3 * n + n * n
    rsv = 32 + 4 * n + n * n
    st = st.astype(np.int64)
    tot = st[:, 0, :6] + st[:, gems:gems + n, :6].sum(1)
    assert (tot[:, :5] == gems_in_play).all() and (tot[:, 5] == 5).all()
    visible = (st[:, 1:25:2, :5].sum(2) != 0).sum(1)
    deck = st[:, 25:31:2, :5].sum((1, 2))
    reserved = (st[:, rsv:rsv + 6 * n:2, :5].sum(2) != 0).sum(1)
    bought = st[:, cards:cards + n, :5].sum((1, 2))
    assert (visible + deck + reserved + bought == 90).all()
    assert st.shape[1] == R


@pytest.mark.parametrize("n", (2, 4))
def test_full_size_rollout_invariants(engines, n):
    """BASELINE config 2 size: 32768 boards; size-independent properties every step."""
    from splendor.env import RolloutBatch, unpack_mask
    B = 32768 if n == 2 else 16384
    rb = RolloutBatch(engines[n], B, seed=0x5EED)
    gip = {2: 4, 3: 5, 4: 7}[n]
    prev_round = engines[n].round(rb.state)
    for t in range(150):
        rb.step()
        m = unpack_mask(rb.mask)
        legal = m[torch.arange(B, device="cuda"), rb.action.long()]
        assert bool(legal.all()), f"illegal action chosen at t={t}"
        r = engines[n].round(rb.state)
        ended = (rb.ended != 0).any(1)
        assert bool(((r == prev_round + 1) | ended).all())
        prev_round = r
        if t % 25 == 0:
            _invariants(n, rb.state.cpu().numpy(), gip)
    assert int(rb.games.sum()) > 0


def test_full_size_first_64_steps_bit_exact(engines):
    """SURVEY §8(d) config 2 check at full size: all 32,768 boards, the first 64 steps (one
    launch of 64 moves, the bench's kernel) against the oracle's loop: every action and end
    vector, every word of every legality mask, final boards, players and game counters."""
    from splendor.env import RolloutBatch
    B, T, seed = 32768, 64, 0x5EED
    ref = O.rollout_run(2, B, T, seed, masks=True)
    rb = RolloutBatch(engines[2], B, seed=seed)
    o = rb.run(T)
    np.testing.assert_array_equal(o["action"].cpu().numpy(), ref["action"])
    np.testing.assert_array_equal(o["ended"].cpu().numpy(), ref["ended"])
    msk = o["mask"].cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(msk, ref["masks"])      # word for word (117 MB at this size)
    np.testing.assert_array_equal(rb.state.cpu().numpy(), ref["state"])
    np.testing.assert_array_equal(rb.player.cpu().numpy(), ref["player"])
    np.testing.assert_array_equal(rb.games.cpu().numpy(), ref["games"])


def test_bad_action_sets_error(engines):
    e, d = engines[2], load("env_2p.npz")
    st = dev(d["state"][:4])
    before = st.clone()
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    e.step(st, dev(np.array([500, -1, 3000, 409], np.int16)), None, None, deterministic=True, err=err)
    assert int(err.item()) == 1
    assert torch.equal(st, before)
