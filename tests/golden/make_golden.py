#!/usr/bin/env python3
"""Golden-vector generator for the Splendor hot path (runs ONLY in the build container).

This script is test infrastructure. It reads the reference sources under
/root/reference as *text*, applies the minimal in-memory patches that SURVEY.md §8c
documents, executes them with tiny numba/colorama shims, and records input/output
vectors into ``tests/golden/*.npz``. Nothing from the reference is written to disk:
only numeric fixtures (states, masks, actions, uniforms, results) are saved.

Patches (all in memory, each mirrors a Numba behaviour that plain NumPy 2 rejects or
a hole in the reference at HEAD):
  P1  SplendorLogicNumba.py:682-683  `_valid_select_noble` is an unfinished stub
      (SyntaxError) -> returns zeros(3) (select-noble never valid).
  P2  SplendorLogicNumba.py:54       np.bool8 (removed in NumPy 2) -> np.bool_.
  P3  SplendorLogicNumba.py:44-46    my_packbits result stored into int8 wraps under Numba
      (255/252/240 -> -1/-4/-16): emulated with an explicit uint8->int8 view.
  P4  SplendorLogicNumba.py:313      int8(999) wraps to -25 under Numba: emulated.
  P5  SplendorLogicNumba.py:284-285  actions 405..408 index give_ids3[40..43] out of
      bounds: defined as "no-op + round counter increment" (pass / select-noble).
Type-rule patches (the deployed reference ran under Numba + NumPy 1.x: it uses np.bool8,
removed in NumPy 2). Under NumPy 2's NEP 50 the plain-Python execution would silently do
float32 arithmetic where the deployed code does float64; these restore the deployed rules:
  P6  MCTS.py:199-219  pick_highest_UCB is @njit: Numba types Ps[a] (f32) * cpuct (f64) as
      f64 -> call it with Ps as float64 and Qs/Ns/cpuct/fpu as Python floats.
  P7  MCTS.py:172      Qs update (plain Python, NumPy 1.x legacy promotion = float64).
  P8  MCTS.py:71       policy-target pruning sqrt(k*Psa*sims) in float64.
  P9  MCTS.py:248      softmax is @njit: Numba types Ps (f32) ** (1./T) (f64) as float64, so
                       the power is taken in float64 (then normalised and cast to float32).
  P10 MCTS.py:185      applyDirNoise under NumPy 1.x scalar rules: float32 Ps[idx] * 0.75 is
                       float64, the mix is float64 and stored into the float32 Ps.
Chance injection (the reference is unseeded):
  np.random.random -> pops the next double of an injected uniform stream.
  np.random.choice(10, k, replace=False) (noble draw, SplendorLogicNumba.py:241) ->
      partial Fisher-Yates driven by the same stream: for i<k: j=i+floor(u*(10-i)).
  np.random.choice(n, p=p) (Coach.random_pick, Coach.py:32) -> numpy's legacy algorithm
      (cdf = cumsum(p) / cdf[-1], searchsorted(cdf, u, 'right')) on one injected uniform;
      checked against numpy's RandomState.choice at start-up.
  np.random.choice(bestAs) (MCTS.py:89, temp-0 tie-break) -> bestAs[floor(u * len)].
  MCTS.rng.random / MCTS.rng.dirichlet (MCTS.py:54, :181) -> the keyed Philox draws of the
      device / oracle (tests/golden/detrand.py), so whole episodes (Coach.executeEpisode)
      and arena games (Arena.playGames) replay with the build's random streams.

Usage:  python tests/golden/make_golden.py [nnet3,train,bigmcts]   (writes tests/golden/*.npz;
        with a list, only those groups: nnet3 / train (round 3), bigmcts (round 6: 2p at 1,600
        and 4p at 400 simulations, hash and peaked networks, tree reuse))
"""
import os
import sys
import types
import math

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)
import detrand  # noqa: E402


# ----------------------------------------------------------------------------- shims
def _install_shims():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden.py needs /root/reference (build container only)")
    numba = types.ModuleType("numba")

    def njit(*a, **k):
        if len(a) == 1 and callable(a[0]) and not k:
            return a[0]
        return lambda f: f
    numba.njit = njit
    numba.jit = njit

    class _T:
        def __getitem__(self, item):
            return self
    for name in ("int8", "uint8", "bool_", "int64", "float32", "float64"):
        setattr(numba, name, _T())
    exp = types.ModuleType("numba.experimental")
    exp.jitclass = lambda spec: (lambda cls: cls)
    numba.experimental = exp
    sys.modules["numba"] = numba
    sys.modules["numba.experimental"] = exp

    colorama = types.ModuleType("colorama")

    class _Blank:
        def __getattr__(self, item):
            return ""
    colorama.Style = colorama.Fore = colorama.Back = _Blank()
    sys.modules["colorama"] = colorama
    np.bool8 = np.bool_  # P2


def _exec_module(name, path, patches=()):
    with open(path, "r", encoding="utf-8") as f:
        src = f.read()
    for old, new in patches:
        assert old in src, f"patch anchor not found in {path}: {old!r}"
        src = src.replace(old, new)
    mod = types.ModuleType(name)
    mod.__file__ = "<in-memory " + os.path.basename(path) + ">"
    pkg = name.rpartition(".")[0]
    if pkg:
        mod.__package__ = pkg
    sys.modules[name] = mod
    exec(compile(src, mod.__file__, "exec"), mod.__dict__)
    return mod


def load_reference():
    _install_shims()
    pkg = types.ModuleType("splendor")
    pkg.__path__ = []
    sys.modules["splendor"] = pkg
    logic = _exec_module("splendor.SplendorLogic", f"{REF}/SplendorLogic.py")
    numba_logic = _exec_module(
        "splendor.SplendorLogicNumba", f"{REF}/SplendorLogicNumba.py",
        patches=[
            ("\tdef _valid_select_noble(player):\n\t\tif \n",
             "\tdef _valid_select_noble(self, player):\n\t\treturn np.zeros(3, dtype=np.int8)\n"),  # P1
            ("num_cards_masked[np.where(scores < score_max)] = 999",
             "num_cards_masked[np.where(scores < score_max)] = np.int8(-25)"),  # P4
        ])

    def my_packbits(array):  # P3
        product = np.multiply(array.astype(np.uint8), numba_logic.mask[:len(array)])
        return np.array([product.sum()], dtype=np.uint64).astype(np.uint8).view(np.int8)[0]
    numba_logic.my_packbits = my_packbits

    Board = numba_logic.Board
    orig_make_move = Board.make_move

    def make_move(self, move, player, deterministic):  # P5
        if move >= 405:
            self.bank[0][6] += 1
            return (player + 1) % self.num_players
        return orig_make_move(self, move, player, deterministic)
    Board.make_move = make_move

    _exec_module("Game", f"{REF}/Game.py")
    game_mod = _exec_module("splendor.SplendorGame", f"{REF}/SplendorGame.py")
    mcts_mod = _exec_module(
        "MCTS", f"{REF}/MCTS.py",
        patches=[
            ("Qs = ((Ns+1) * Qs + v[0]) / (Ns+2)",
             "Qs = ((Ns+1) * float(Qs) + float(v[0])) / (Ns+2)"),  # P7
            ("Psas   = [self.nodes_data[s][2][a] for a",
             "Psas   = [float(self.nodes_data[s][2][a]) for a"),  # P8
            ("result = Ps ** (1. / softmax_temp)",
             "result = np.asarray(Ps, dtype=np.float64) ** (1. / softmax_temp)"),  # P9
            ("Ps[idx] = (0.75 * Ps[idx]) + (0.25 * dir_values[dir_idx])",
             "Ps[idx] = (0.75 * float(Ps[idx])) + (0.25 * float(dir_values[dir_idx]))"),  # P10
        ])
    orig_ucb = mcts_mod.pick_highest_UCB

    def pick_highest_UCB(Es, Vs, Ps, Ns, Qsa, Nsa, Qs, cpuct, forced_playouts, n_iter, fpu):  # P6
        return orig_ucb(Es, Vs, np.asarray(Ps, dtype=np.float64), float(Ns), Qsa, Nsa,
                        float(Qs), float(cpuct), forced_playouts, n_iter, float(fpu))
    mcts_mod.pick_highest_UCB = pick_highest_UCB
    return logic, numba_logic, game_mod, mcts_mod


# ------------------------------------------------------------------ chance injection
class UniformStream:
    """Replaces np.random.random / np.random.choice(replace=False) while active."""

    def __init__(self):
        self.src = None
        self.used = []
        self.pick = None      # source of Coach.random_pick's uniform
        self.tie = None       # source of the temp-0 tie-break uniform

    def set_source(self, rng):
        self.src = rng
        self.used = []

    def random(self, *a, **k):
        assert not a and not k
        u = float(self.src.random())
        self.used.append(u)
        return u

    def choice(self, a, size=None, replace=True, p=None):
        if p is not None:                       # Coach.random_pick: legacy choice with p
            assert size is None and isinstance(a, (int, np.integer))
            return legacy_choice_p(int(a), p, self.pick.random())
        if not isinstance(a, (int, np.integer)):   # MCTS.py:89 tie-break over bestAs
            assert size is None
            a = np.asarray(a)
            return a[int(self.tie.random() * len(a))]
        assert replace is False
        perm = list(range(int(a)))
        for i in range(int(size)):
            u = self.random()
            j = i + int(math.floor(u * (int(a) - i)))
            perm[i], perm[j] = perm[j], perm[i]
        return np.array(perm[:size], dtype=np.int64)


STREAM = UniformStream()


def legacy_choice_p(n, p, u):
    """numpy RandomState.choice(n, p=p) given its one uniform draw u (mtrand.pyx: cdf =
    p.cumsum(); cdf /= cdf[-1]; cdf.searchsorted(u, side='right'))."""
    p = np.asarray(p, dtype=np.float64)
    assert len(p) == n and np.all(p >= 0) and abs(p.sum() - 1.0) <= math.sqrt(np.finfo(np.float64).eps)
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return int(np.searchsorted(cdf, u, side="right"))


def _check_legacy_choice():
    rng = np.random.default_rng(5)
    for t in range(200):
        p = rng.random(409) * (rng.random(409) < 0.1)
        p[rng.integers(409)] += 1e-3
        p = list(p / p.sum())
        a = np.random.RandomState(t).choice(409, p=p)
        u = np.random.RandomState(t).random_sample()
        assert a == legacy_choice_p(409, p, u), "legacy choice restatement mismatch"


class InjectedRng:
    """MCTS.rng replacement (MCTS.py:40): random() -> keyed full/fast draw, dirichlet() ->
    the build's keyed Dirichlet sampler (detrand.dirichlet)."""

    def __init__(self):
        self.full = None          # (seed, board, stream) of the next rng.random()
        self.dir = None           # (seed, board, stream) of the next rng.dirichlet()

    def random(self):
        return detrand.uniform(*self.full, 0)

    def dirichlet(self, alphas):
        alphas = list(alphas)
        assert all(a == alphas[0] for a in alphas)
        return np.array(detrand.dirichlet(float(alphas[0]), *self.dir, len(alphas)), dtype=np.float64)


def _patch_np_random():
    np.random.random = STREAM.random
    np.random.choice = STREAM.choice


# ----------------------------------------------------------------------- fake NN
M64 = (1 << 64) - 1


def fnv1a64(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for b in data:
        h ^= b
        h = (h * 0x100000001B3) & M64
    return h


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def fake_predict(state, valids, n_players):
    """Deterministic stand-in for SplendorNNet used for search-parity fixtures.
    pi[a] = (1 + (splitmix64(h + a) >> 40)) * 2^-24 for valid a (exact in f32), 0 else.
    v[i]  = (splitmix64(h ^ (0xA5A5 + i)) >> 40) * 2^-23 - 1  (exact in f32)."""
    h = fnv1a64(np.ascontiguousarray(state).view(np.uint8).tobytes())
    pi = np.zeros(len(valids), dtype=np.float32)
    for a in np.flatnonzero(valids):
        pi[a] = np.float32((1 + (splitmix64((h + int(a)) & M64) >> 40)) * 2.0 ** -24)
    v = np.array([np.float32((splitmix64(h ^ (0xA5A5 + i)) >> 40) * 2.0 ** -23 - 1.0)
                  for i in range(n_players)], dtype=np.float32)
    return pi, v


class FakeNNet:
    def __init__(self, n):
        self.n = n

    def predict(self, board, valid_actions):
        return fake_predict(board, np.asarray(valid_actions, dtype=bool), self.n)


# ------------------------------------------------------------------- env fixtures
def env_fixtures(numba_logic, n_players, n_games, seed, det_every=3):
    Board = numba_logic.Board
    game_rng = np.random.default_rng(seed)
    rec = {k: [] for k in ("state", "player", "canon", "mask_canon", "mask_player",
                           "ended", "scores", "round", "action", "next_state",
                           "next_player", "next_ended", "u_off", "u_len")}
    uni = []
    det = {k: [] for k in ("src", "action", "next_state", "next_player")}
    init = {"uniforms": [], "state": []}
    for g in range(n_games):
        STREAM.set_source(np.random.default_rng([seed, g, 1]))
        b = Board(n_players)          # __init__ -> init_game (24 card uniforms + nobles)
        init["uniforms"].append(np.array(STREAM.used, dtype=np.float64))
        init["state"].append(b.get_state().copy())
        state = b.get_state().copy()
        player = 0
        scratch = Board(n_players)
        for ply in range(400):
            idx = len(rec["state"])
            rec["state"].append(state.copy())
            rec["player"].append(player)
            scratch.copy_state(state, True)
            if player != 0:
                scratch.swap_players(player)
            canon = scratch.get_state().copy()
            rec["canon"].append(canon)
            scratch.copy_state(canon, True)
            mc = scratch.valid_moves(0).astype(np.uint8)
            rec["mask_canon"].append(mc)
            scratch.copy_state(state, True)
            mp = scratch.valid_moves(player).astype(np.uint8)
            rec["mask_player"].append(mp)
            scratch.copy_state(state, True)
            rec["ended"].append(scratch.check_end_game().astype(np.float32))
            rec["scores"].append([scratch.get_score(p) for p in range(n_players)])
            rec["round"].append(int(scratch.get_round()))
            # deterministic in-tree steps from the canonical board (MCTS.py:227-235)
            if ply % det_every == 0:
                for a in np.flatnonzero(mc):
                    scratch.copy_state(canon, True)
                    nxt = scratch.make_move(int(a), 0, True)
                    if nxt != 0:
                        scratch.swap_players(nxt)
                    det["src"].append(idx)
                    det["action"].append(int(a))
                    det["next_state"].append(scratch.get_state().copy())
                    det["next_player"].append(nxt)
            # real move with chance on the non-canonical board (Coach.py:86)
            valid = np.flatnonzero(mp)
            a = int(valid[game_rng.integers(len(valid))])
            STREAM.set_source(np.random.default_rng([seed, g, 2, ply]))
            scratch.copy_state(state, True)
            nxt = scratch.make_move(a, player, False)
            rec["action"].append(a)
            rec["next_state"].append(scratch.get_state().copy())
            rec["next_player"].append(nxt)
            rec["u_off"].append(len(uni))
            rec["u_len"].append(len(STREAM.used))
            uni.extend(STREAM.used)
            state = scratch.get_state().copy()
            player = nxt
            scratch.copy_state(state, True)
            ended = scratch.check_end_game().astype(np.float32)
            rec["next_ended"].append(ended)
            if ended.any():
                break
    out = {}
    for k, v in rec.items():
        out[k] = np.array(v)
    out["uniforms"] = np.array(uni, dtype=np.float64)
    for k, v in det.items():
        out["det_" + k] = np.array(v)
    out["init_state"] = np.array(init["state"])
    out["init_uniforms"] = np.array(init["uniforms"])
    return out


def crafted_end_cases(numba_logic, n_players):
    """Known-answer end-of-game vectors (debug.py:41-42 tie case, 3p [15,15,3], cap)."""
    Board = numba_logic.Board
    R = 32 + 10 * n_players + n_players * n_players
    base = 32 + n_players
    cards0 = base + n_players + n_players * (n_players + 1)
    states, ends = [], []
    rng = np.random.default_rng(99 + n_players)
    cases = []
    if n_players == 2:
        cases += [([15, 15], [14, 12]), ([15, 15], [12, 12]), ([16, 15], [3, 3]), ([15, 3], [9, 9]),
                  ([3, 3], [1, 2]), ([14, 14], [5, 6])]
    elif n_players == 3:
        cases += [([15, 15, 3], [5, 6, 1]), ([15, 15, 15], [4, 4, 9]), ([15, 15, 3], [6, 6, 6]),
                  ([17, 15, 3], [1, 1, 1])]
    else:
        cases += [([15, 15, 3, 0], [5, 6, 1, 0]), ([15, 14, 15, 15], [4, 4, 4, 9]),
                  ([16, 2, 2, 2], [3, 3, 3, 3])]
    for rnd_mode in ("mid", "cap", "odd"):
        for scores, ncards in cases:
            st = np.zeros((R, 7), dtype=np.int8)
            for p in range(n_players):
                st[cards0 + p, 6] = scores[p]
                # distribute card counts over colours
                c = ncards[p]
                for col in range(5):
                    take = min(c, int(rng.integers(0, 4)) if col < 4 else c)
                    st[cards0 + p, col] = take
                    c -= take
            r = {"mid": 10 * n_players, "cap": 62 * n_players, "odd": 10 * n_players + 1}[rnd_mode]
            st[0, 6] = np.array([r], dtype=np.uint8).view(np.int8)[0]
            b = Board(n_players)
            b.copy_state(st, True)
            states.append(st)
            ends.append(b.check_end_game().astype(np.float32))
    return {"state": np.array(states), "ended": np.array(ends)}


# ------------------------------------------------------------------ MCTS fixtures
def mcts_fixtures(game_mod, mcts_mod, numba_logic, n_players, seed, cases):
    """Single-move searches from seeded positions + a multi-move game with tree reuse.
    Dirichlet off (rng-dependent); forced playouts exercised (deterministic)."""
    Game = game_mod.SplendorGame
    out = {k: [] for k in ("root", "sims", "cpuct", "fpu", "forced", "counts", "qsa", "probs",
                           "q", "ns", "case")}
    seq = {k: [] for k in ("root", "counts", "probs", "q", "action", "uoff", "ulen", "move", "player")}
    seq_uni = []
    Board = numba_logic.Board
    game_rng = np.random.default_rng(seed)
    # collect a pool of positions from random play
    pool = []
    STREAM.set_source(np.random.default_rng([seed, 7]))
    b = Board(n_players)
    state, player = b.get_state().copy(), 0
    scratch = Board(n_players)
    while len(pool) < 40:
        scratch.copy_state(state, True)
        if player != 0:
            scratch.swap_players(player)
        pool.append(scratch.get_state().copy())
        scratch.copy_state(state, True)
        v = np.flatnonzero(scratch.valid_moves(player))
        STREAM.set_source(np.random.default_rng([seed, 8, len(pool)]))
        scratch.copy_state(state, True)
        player = scratch.make_move(int(v[game_rng.integers(len(v))]), player, False)
        state = scratch.get_state().copy()
        scratch.copy_state(state, True)
        if scratch.check_end_game().any():
            STREAM.set_source(np.random.default_rng([seed, 9, len(pool)]))
            b = Board(n_players)
            state, player = b.get_state().copy(), 0
    for ci, (sims, cpuct, fpu, forced) in enumerate(cases):
        for pi_, root in enumerate(pool[ci::len(cases)][:6]):
            g = Game(n_players)
            args = {"numMCTSSims": sims, "cpuct": cpuct, "fpu": fpu, "prob_fullMCTS": 1.0,
                    "ratio_fullMCTS": 5, "forced_playouts": forced, "no_mem_optim": False,
                    "dirichletAlpha": 0.0, "temperature": [1.25, 0.8]}
            m = mcts_mod.MCTS(g, FakeNNet(n_players), _DotDict(args), dirichlet_noise=False)
            probs, q, full = m.getActionProb(root.copy(), temp=1, force_full_search=True)
            s = g.stringRepresentation(root)
            node = m.nodes_data[s]
            out["root"].append(root.copy())
            out["sims"].append(sims)
            out["cpuct"].append(cpuct)
            out["fpu"].append(fpu)
            out["forced"].append(int(forced))
            out["counts"].append(np.asarray(node[5], dtype=np.int64))
            out["qsa"].append(np.asarray(node[4], dtype=np.float64))
            out["probs"].append(np.asarray(probs, dtype=np.float64))
            out["q"].append(np.asarray(q, dtype=np.float64))
            out["ns"].append(int(node[3]))
            out["case"].append(ci)
    # multi-move self-play with tree persistence; action = first argmax of counts,
    # real step with injected chance (mirrors Coach.executeEpisode minus sampling)
    g = Game(n_players)
    args = {"numMCTSSims": 50, "cpuct": 2.5, "fpu": 0.3, "prob_fullMCTS": 1.0,
            "ratio_fullMCTS": 5, "forced_playouts": False, "no_mem_optim": False,
            "dirichletAlpha": 0.0, "temperature": [1.25, 0.8]}
    m = mcts_mod.MCTS(g, FakeNNet(n_players), _DotDict(args), dirichlet_noise=False)
    STREAM.set_source(np.random.default_rng([seed, 11]))
    board = g.getInitBoard().copy()
    seq["init_uniforms"] = np.array(STREAM.used, dtype=np.float64)
    seq["init_state"] = board.copy()
    cur = 0
    for move in range(30):
        canon = g.getCanonicalForm(board, cur).copy()
        probs, q, full = m.getActionProb(canon, temp=1, force_full_search=True)
        s = g.stringRepresentation(canon)
        counts = np.asarray(m.nodes_data[s][5], dtype=np.int64)
        a = int(np.argmax(counts))
        seq["root"].append(canon)
        seq["counts"].append(counts)
        seq["probs"].append(np.asarray(probs, dtype=np.float64))
        seq["q"].append(np.asarray(q, dtype=np.float64))
        seq["action"].append(a)
        seq["player"].append(cur)
        seq["move"].append(move)
        STREAM.set_source(np.random.default_rng([seed, 12, move]))
        board, cur = g.getNextState(board, cur, a)
        board = board.copy()
        seq["uoff"].append(len(seq_uni))
        seq["ulen"].append(len(STREAM.used))
        seq_uni.extend(STREAM.used)
        if g.getGameEnded(board, cur).any():
            break
    res = {k: np.array(v) for k, v in out.items()}
    for k, v in seq.items():
        res["seq_" + k] = np.array(v)
    res["seq_uniforms"] = np.array(seq_uni, dtype=np.float64)
    return res


class PeakedNNet(FakeNNet):
    """The peaked hash network (oracle `or_fake_predict` mode 1, device `HashEvaluator(mode=1)`)
    restated: w_a = 1 + (splitmix64(h + a) >> 40) over the legal actions, pi[a] = (w_a / max w)^256
    by eight squarings in float64, stored float32 (one or a few actions dominate, many are exactly
    0); v[i] = +-(1 - (splitmix64(h ^ (0xA5A5 + i)) >> 40) * 2^-30), + for player 0. It grows
    trees as deep as the benchmark's random-init SplendorNNet (leaf depths in the tens)."""

    def predict(self, board, valid_actions):
        valids = np.asarray(valid_actions, dtype=bool)
        h = fnv1a64(np.ascontiguousarray(board).view(np.uint8).tobytes())
        w = {int(a): float(1 + (splitmix64((h + int(a)) & M64) >> 40)) for a in np.flatnonzero(valids)}
        wmax = max(w.values())
        pi = np.zeros(len(valids), dtype=np.float32)
        for a, wa in w.items():
            x = wa / wmax
            for _ in range(8):
                x = x * x
            pi[a] = np.float32(x)
        v = np.array([np.float32((1.0 if i == 0 else -1.0) *
                                 (1.0 - (splitmix64(h ^ (0xA5A5 + i)) >> 40) * 2.0 ** -30))
                      for i in range(self.n)], dtype=np.float32)
        return pi, v


def _track_leaf_depths(m):
    """Wraps MCTS.search (the recursion resolves self.search through the instance) to record,
    per simulation, the number of edges from the root to the node it ends at (a new leaf or a
    terminal node): the oracle's or_depth_stats / the device's depth_sum definition."""
    depths, st = [], {"d": 0, "max": 0}
    orig = m.search

    def search(*a, **k):
        st["d"] += 1
        st["max"] = max(st["max"], st["d"])
        try:
            return orig(*a, **k)
        finally:
            st["d"] -= 1
            if st["d"] == 0:
                depths.append(st["max"] - 1)
                st["max"] = 0
    m.search = search
    return depths


def big_mcts_fixtures(game_mod, mcts_mod, numba_logic, n, seed, sims, n_roots, n_peaked, seq_moves):
    """Round 6: the reference's MCTS (MCTS.py:45-97, 99-177, 199-219) at the large budgets of
    BASELINE configs 4 (2p, numMCTSSims 1,600) and 5 (4p, 400), genbu.pt's cpuct 2.5 / fpu 0.3:
    n_roots single searches under the hash network (mode 0) from positions spread over random
    games, n_peaked more under the peaked network (mode 1: deep trees), and one multi-move game
    with tree reuse (the first arg-max of the counts is played, chance injected). Dirichlet off,
    forced playouts off, every search full (force_full_search, as mcts_fixtures)."""
    Game = game_mod.SplendorGame
    Board = numba_logic.Board
    game_rng = np.random.default_rng(seed)
    pool = []
    STREAM.set_source(np.random.default_rng([seed, 7]))
    b = Board(n)
    state, player = b.get_state().copy(), 0
    scratch = Board(n)
    while len(pool) < 120:
        scratch.copy_state(state, True)
        if player != 0:
            scratch.swap_players(player)
        pool.append(scratch.get_state().copy())
        scratch.copy_state(state, True)
        v = np.flatnonzero(scratch.valid_moves(player))
        STREAM.set_source(np.random.default_rng([seed, 8, len(pool)]))
        scratch.copy_state(state, True)
        player = scratch.make_move(int(v[game_rng.integers(len(v))]), player, False)
        state = scratch.get_state().copy()
        scratch.copy_state(state, True)
        if scratch.check_end_game().any():
            STREAM.set_source(np.random.default_rng([seed, 9, len(pool)]))
            b = Board(n)
            state, player = b.get_state().copy(), 0
    args = {"numMCTSSims": sims, "cpuct": 2.5, "fpu": 0.3, "prob_fullMCTS": 1.0, "ratio_fullMCTS": 5,
            "forced_playouts": False, "no_mem_optim": False, "dirichletAlpha": 0.0,
            "temperature": [1.25, 0.8]}
    out = {k: [] for k in ("root", "mode", "counts", "qsa", "probs", "q", "ns", "nodes", "depth")}
    step = len(pool) // (n_roots + n_peaked)
    roots = pool[::step][:n_roots + n_peaked]
    for i, root in enumerate(roots):
        mode = 0 if i < n_roots else 1
        g = Game(n)
        net = FakeNNet(n) if mode == 0 else PeakedNNet(n)
        m = mcts_mod.MCTS(g, net, _DotDict(args), dirichlet_noise=False)
        depths = _track_leaf_depths(m)
        probs, q, _ = m.getActionProb(root.copy(), temp=1, force_full_search=True)
        node = m.nodes_data[g.stringRepresentation(root)]
        out["root"].append(root.copy())
        out["mode"].append(mode)
        out["nodes"].append(len(m.nodes_data))
        out["depth"].append([sum(depths), max(depths), len(depths)])
        out["counts"].append(np.asarray(node[5], dtype=np.int64))
        out["qsa"].append(np.asarray(node[4], dtype=np.float64))
        out["probs"].append(np.asarray(probs, dtype=np.float64))
        out["q"].append(np.asarray(q, dtype=np.float64))
        out["ns"].append(int(node[3]))
        print(f"  {n}p {sims} sims root {i} mode {mode}: {int((out['counts'][-1] > 0).sum())} visited edges, "
              f"max N {int(out['counts'][-1].max())}, {len(m.nodes_data)} nodes, leaf depth mean "
              f"{sum(depths) / len(depths):.1f} max {max(depths)}", flush=True)
    seq = {k: [] for k in ("root", "counts", "probs", "q", "action", "uoff", "ulen")}
    seq_uni = []
    g = Game(n)
    m = mcts_mod.MCTS(g, FakeNNet(n), _DotDict(args), dirichlet_noise=False)
    STREAM.set_source(np.random.default_rng([seed, 11]))
    board = g.getInitBoard().copy()
    init_uniforms, init_state = np.array(STREAM.used, dtype=np.float64), board.copy()
    cur = 0
    for move in range(seq_moves):
        canon = g.getCanonicalForm(board, cur).copy()
        probs, q, _ = m.getActionProb(canon, temp=1, force_full_search=True)
        counts = np.asarray(m.nodes_data[g.stringRepresentation(canon)][5], dtype=np.int64)
        a = int(np.argmax(counts))
        seq["root"].append(canon)
        seq["counts"].append(counts)
        seq["probs"].append(np.asarray(probs, dtype=np.float64))
        seq["q"].append(np.asarray(q, dtype=np.float64))
        seq["action"].append(a)
        STREAM.set_source(np.random.default_rng([seed, 12, move]))
        board, cur = g.getNextState(board, cur, a)
        board = board.copy()
        seq["uoff"].append(len(seq_uni))
        seq["ulen"].append(len(STREAM.used))
        seq_uni.extend(STREAM.used)
        if g.getGameEnded(board, cur).any():
            break
    res = {k: np.array(v) for k, v in out.items()}
    for k, v in seq.items():
        res["seq_" + k] = np.array(v)
    res["seq_uniforms"] = np.array(seq_uni, dtype=np.float64)
    res["seq_init_uniforms"] = init_uniforms
    res["seq_init_state"] = init_state
    res["sims"] = np.array(sims)
    res["cpuct"] = np.array(2.5)
    res["fpu"] = np.array(0.3)
    return res


class _DotDict(dict):
    def __getattr__(self, k):
        return self[k]


def fake_nn_vectors(numba_logic, n_players, states):
    pis, vs, masks = [], [], []
    b = numba_logic.Board(n_players)
    for st in states:
        b.copy_state(st, True)
        m = b.valid_moves(0)
        pi, v = fake_predict(st, m, n_players)
        pis.append(pi)
        vs.append(v)
        masks.append(m.astype(np.uint8))
    return {"state": np.array(states), "mask": np.array(masks), "pi": np.array(pis),
            "v": np.array(vs)}


def deterministic_weights(state_dict):
    """Assign every tensor of a SplendorNNet state_dict a closed-form value pattern (by
    sorted key order) so an independent re-implementation can load identical weights."""
    import torch
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


def nnet_fixture(n_players, boards):
    import torch
    _exec_module("splendor.SplendorNNet", f"{REF}/SplendorNNet.py")
    mod = sys.modules["splendor.SplendorNNet"]

    class _G:
        num_players = n_players
        def getBoardSize(self):
            return (32 + 10 * n_players + n_players * n_players, 7)
        def getActionSize(self):
            return 409
        def getMaxScoreDiff(self):
            return 15
    net = mod.SplendorNNet(_G(), {"nn_version": 1, "dropout": 0.3}, use_token_exchange=True)
    sd = deterministic_weights(net.state_dict())
    net.load_state_dict(sd)
    net.eval()
    b = torch.from_numpy(boards.astype(np.float32))
    valid = torch.from_numpy(np.stack([(np.arange(409) % (3 + i)) != 0 for i in range(len(boards))]))
    with torch.no_grad():
        lp, v, sdf = net(b, valid)
    return {"boards": boards, "valid": valid.numpy(), "log_pi": lp.numpy(), "v": v.numpy(),
            "sdiff": sdf.numpy(), "keys": np.array(sorted(sd)),
            "n_params": np.array(sum(p.numel() for p in net.parameters()))}



def load_trainer():
    """GenericNNetWrapper + splendor/NNet.py (the reference's training consumer) with an
    onnxruntime stub (only predict's onnx mode and export use it; train never does)."""
    import importlib.machinery
    ort = types.ModuleType("onnxruntime")
    ort.__spec__ = importlib.machinery.ModuleSpec("onnxruntime", None)
    ort.SessionOptions = ort.InferenceSession = object
    sys.modules["onnxruntime"] = ort
    _exec_module("utils", f"{REF}/utils.py")
    _exec_module("NeuralNet", f"{REF}/NeuralNet.py")
    _exec_module("GenericNNetWrapper", f"{REF}/GenericNNetWrapper.py")
    if "splendor.SplendorNNet" not in sys.modules:
        _exec_module("splendor.SplendorNNet", f"{REF}/SplendorNNet.py")
    return _exec_module("splendor.NNet", f"{REF}/NNet.py")


def train_fixture(nnet_mod, n_players, canon, masks, E, bs, epochs, lr, dropout, seed):
    """GenericNNetWrapper.train (:43-139) on CPU over E synthetic examples built from real
    positions (board = a recorded canonical state, valids its mask, pi random over the
    valids, winner +-1, scdiff in [-20, 20], surprise random), with the reference's
    SplendorNNet under deterministic_weights and every np.random.choice batch (:70)
    injected from a seeded RandomState and recorded. Records each step's four losses
    (:94-98) and the final state_dict (parameters and BatchNorm running statistics).
    dropout > 0: torch.manual_seed(seed) right before train, so a restatement that draws
    its dropout masks in the reference's order on the CPU generator sees the same masks."""
    import torch
    rs = np.random.RandomState(seed)
    idx = rs.randint(0, len(canon), E)
    boards = canon[idx].astype(np.int8)
    valids = masks[idx].astype(bool)
    pis = np.where(valids, rs.random_sample(valids.shape), 0.0).astype(np.float32)
    pis /= pis.sum(1, keepdims=True)
    w = np.where(rs.random_sample(E) < 0.5, 1.0, -1.0)
    winner = (np.stack([w] + [-w / (n_players - 1)] * (n_players - 1), 1)).astype(np.float32)
    scdiff = rs.randint(-20, 21, (E, n_players)).astype(np.int8)
    surprise = rs.random_sample((E, n_players)).astype(np.float32)
    examples = [(boards[i], pis[i], winner[i], scdiff[i], valids[i], surprise[i]) for i in range(E)]

    class _G:
        num_players = n_players
        def getBoardSize(self):
            return (32 + 10 * n_players + n_players * n_players, 7)
        def getActionSize(self):
            return 409
        def getMaxScoreDiff(self):
            return 15
    args = {"nn_version": 1, "dropout": dropout, "learn_rate": lr, "batch_size": bs, "epochs": epochs,
            "vl_weight": 10.0, "surprise_weight": False, "no_compression": True}
    w_ = nnet_mod.NNetWrapper(_G(), args)
    sd0 = deterministic_weights(w_.nnet.state_dict())
    w_.nnet.load_state_dict(sd0)
    ids_log, loss_log = [], []
    orig_choice = np.random.choice

    def choice(a, size=None, replace=True, p=None):
        assert isinstance(a, int) and size == bs and replace is False and p is None
        ids = rs.permutation(a)[:size]
        ids_log.append(ids.copy())
        return ids
    wrapped = {}
    for name in ("loss_pi", "loss_v", "loss_scdiff_cdf", "loss_scdiff_pdf"):
        f = getattr(w_, name)
        wrapped[name] = f

        def rec(t, o, _f=f, _n=name):
            r = _f(t, o)
            if _n == "loss_pi":
                loss_log.append([])
            loss_log[-1].append(float(r.item()))
            return r
        setattr(w_, name, rec)
    np.random.choice = choice
    try:
        torch.manual_seed(seed)
        w_.train(examples)
    finally:
        np.random.choice = orig_choice
    sd = w_.nnet.state_dict()
    out = {"boards": boards, "valids": valids, "pi": pis, "winner": winner, "scdiff": scdiff,
           "surprise": surprise, "sample_ids": np.array(ids_log, dtype=np.int64),
           "losses": np.array(loss_log, dtype=np.float64),
           "args": np.array([E, bs, epochs, lr, dropout, 10.0, seed], dtype=np.float64),
           "keys": np.array(sorted(sd))}
    for k in sorted(sd):
        out["p:" + k] = sd[k].detach().cpu().numpy()
    return out

# ------------------------------------------------------------- noise / episode / arena
ST_FULL, ST_DIR, ST_PICK, ST_MOVE, ST_DEAL, ST_BEST = (1 << 24), (2 << 24), (3 << 24), (4 << 24), (5 << 24), (6 << 24)
GEM_TOTAL = {2: 4, 3: 5, 4: 7}


class FakeNNetC(FakeNNet):
    """FakeNNet with the NeuralNet constructor signature (Coach.py:44 builds a second one);
    neg=True negates v (a second, different 'network' for arena games)."""

    def __init__(self, game, args=None, neg=False):
        super().__init__(game.num_players)
        self.args = args or {}
        self.neg = neg

    def predict(self, board, valid_actions):
        pi, v = super().predict(board, valid_actions)
        return (pi, -v) if self.neg else (pi, v)


def wide_roots(numba_logic, n, states):
    """Canonical positions with the widest action sets: player 0 holds 2 gems of every colour
    (10 tokens: every exchange family is open), the bank holds the rest of each colour and 5
    gold. 4p positions reach 229 legal actions (> 3 x 64)."""
    Board = numba_logic.Board
    b = Board(n)
    out = []
    for st in states:
        s_ = st.copy()
        for p in range(n):
            s_[32 + n + p, :6] = 0
        s_[32 + n, :5] = 2
        s_[0, :5] = GEM_TOTAL[n] - 2
        s_[0, 5] = 5
        b.copy_state(s_, True)
        out.append((int(b.valid_moves(0).sum()), s_))
    out.sort(key=lambda x: -x[0])
    return [x[1] for x in out]


def noise_fixtures(game_mod, mcts_mod, numba_logic, n, states, seed):
    """softmax(Ps, T0) -> applyDirNoise -> normalise (MCTS.py:141-144) on raw network priors,
    and on stored (normalised) priors (:150-154), with injected Dirichlet vectors."""
    Game = game_mod.SplendorGame
    Board = numba_logic.Board
    b = Board(n)
    rec = {k: [] for k in ("ps_in", "vs", "dir", "temp0", "alpha", "key", "ps_out", "stored")}
    for i, st in enumerate(states):
        b.copy_state(st, True)
        vs = b.valid_moves(0)
        raw, _ = fake_predict(st, vs, n)
        for j, (t0, alpha, stored) in enumerate(((1.25, 0.3, False), (1.0, 0.3, False), (1.25, 0.2, True),
                                                 (0.8, 1.5, True))):
            ps = raw.copy()
            if stored:
                mcts_mod.normalise(ps)
            key = (seed, i, ST_DIR | j)
            dirv = np.array(detrand.dirichlet(alpha, *key, int(vs.sum())))
            g = Game(n)
            m = mcts_mod.MCTS(g, FakeNNet(n), _DotDict({"dirichletAlpha": alpha, "temperature": [t0, 0.8]}),
                              dirichlet_noise=True)
            m.rng = InjectedRng()
            m.rng.dir = key
            pin = ps.copy()
            P = mcts_mod.softmax(ps, t0)
            m.applyDirNoise(P, vs)
            mcts_mod.normalise(P)
            d409 = np.zeros(409)
            d409[:len(dirv)] = dirv
            rec["ps_in"].append(pin)
            rec["vs"].append(vs.astype(np.uint8))
            rec["dir"].append(d409)
            rec["temp0"].append(t0)
            rec["alpha"].append(alpha)
            rec["key"].append(np.array(key, dtype=np.uint64))
            rec["ps_out"].append(np.asarray(P, dtype=np.float32))
            rec["stored"].append(int(stored))
    return {k: np.array(v) for k, v in rec.items()}


def noise_search_fixtures(game_mod, mcts_mod, n, roots, seed, cases):
    """Full searches with root Dirichlet noise (MCTS.py:58-59), two searches per tree from
    the same root (the second re-noises the stored priors, :150-154). Tree t of case c has
    board id 100*c + t; search s (1, 2) draws its noise from (seed, board, ST_DIR | s)."""
    Game = game_mod.SplendorGame
    out = {k: [] for k in ("root", "case", "board", "sims", "cpuct", "fpu", "alpha", "temp0", "forced",
                           "counts1", "qsa1", "probs1", "q1", "counts2", "qsa2", "probs2", "q2")}
    for ci, (sims, cpuct, fpu, alpha, t0, forced) in enumerate(cases):
        for t, root in enumerate(roots):
            g = Game(n)
            args = {"numMCTSSims": sims, "cpuct": cpuct, "fpu": fpu, "prob_fullMCTS": 1.0,
                    "ratio_fullMCTS": 5, "forced_playouts": forced, "no_mem_optim": False,
                    "dirichletAlpha": alpha, "temperature": [t0, 0.8]}
            m = mcts_mod.MCTS(g, FakeNNet(n), _DotDict(args), dirichlet_noise=True)
            m.rng = InjectedRng()
            board = 100 * ci + t
            s = g.stringRepresentation(root)
            for k in (1, 2):
                m.rng.dir = (seed, board, ST_DIR | k)
                probs, q, _ = m.getActionProb(root.copy(), temp=1, force_full_search=True)
                node = m.nodes_data[s]
                out[f"counts{k}"].append(np.array(node[5], dtype=np.int64, copy=True))
                out[f"qsa{k}"].append(np.array(node[4], dtype=np.float64, copy=True))
                out[f"probs{k}"].append(np.asarray(probs, dtype=np.float64))
                out[f"q{k}"].append(np.asarray(q, dtype=np.float64))
            out["root"].append(root.copy())
            out["case"].append(ci)
            out["board"].append(board)
            for key, val in (("sims", sims), ("cpuct", cpuct), ("fpu", fpu), ("alpha", alpha),
                             ("temp0", t0), ("forced", int(forced))):
                out[key].append(val)
    return {k: np.array(v) for k, v in out.items()}


def load_coach():
    stub = types.ModuleType("Arena")
    stub.Arena = object                      # executeEpisode does not use the Arena
    sys.modules["Arena"] = stub
    mod = _exec_module("Coach", f"{REF}/Coach.py")
    del sys.modules["Arena"]
    return mod


def episode_fixtures(game_mod, coach_mod, n, seed, boards, args):
    """Coach.executeEpisode (Coach.py:50-100), one game per board id, every random draw
    injected from the build's keyed streams (move k of a game: full/fast draw ST_FULL|k,
    Dirichlet ST_DIR|k+1, action pick ST_PICK|k+1, chance ST_MOVE|k+1; deal ST_DEAL|0)."""
    Game = game_mod.SplendorGame
    ex = {k: [] for k in ("board", "pi", "winner", "scdiff", "valids", "surprise", "game")}
    games = {k: [] for k in ("board_id", "moves", "n_examples", "actions")}
    for gi, gb in enumerate(boards):
        STREAM.set_source(np.random.default_rng([seed, gb]))       # constructor's deal (unused)
        g = Game(n)
        c = coach_mod.Coach(g, FakeNNetC(g), _DotDict(args))
        rng = InjectedRng()
        c.mcts.rng = rng
        st = {"k": 0}
        actions = []
        orig_gap, orig_next = c.mcts.getActionProb, g.getNextState

        def gap(canon, temp=1, force_full_search=False, bias=None, _gb=gb):
            k = st["k"]
            rng.full = (seed, _gb, ST_FULL | k)
            rng.dir = (seed, _gb, ST_DIR | (k + 1))
            r = orig_gap(canon, temp=temp, force_full_search=force_full_search, bias=bias)
            STREAM.pick = detrand.Stream(seed, _gb, ST_PICK | (k + 1))
            STREAM.set_source(detrand.Stream(seed, _gb, ST_MOVE | (k + 1)))
            st["k"] = k + 1
            return r

        def nxt(board, player, action, deterministic=False):
            actions.append(int(action))
            return orig_next(board, player, action, deterministic)
        c.mcts.getActionProb = gap
        g.getNextState = nxt
        STREAM.set_source(detrand.Stream(seed, gb, ST_DEAL | 0))
        out = c.executeEpisode()
        for x in out:
            ex["board"].append(np.asarray(x[0], dtype=np.int8))
            ex["pi"].append(np.asarray(x[1], dtype=np.float32))
            ex["winner"].append(np.asarray(x[2], dtype=np.float32))
            ex["scdiff"].append(np.asarray(x[3], dtype=np.int32))
            ex["valids"].append(np.asarray(x[4], dtype=np.uint8))
            ex["surprise"].append(np.asarray(x[5], dtype=np.float64))
            ex["game"].append(gi)
        games["board_id"].append(gb)
        games["moves"].append(st["k"])
        games["n_examples"].append(len(out))
        games["actions"].append(np.array(actions + [-1] * (400 - len(actions)), dtype=np.int16))
    res = {k: np.array(v) for k, v in ex.items()}
    res.update({"game_" + k: np.array(v) for k, v in games.items()})
    for k, v in args.items():
        res["arg_" + k] = np.array(v)
    res["seed"] = np.array(seed, dtype=np.uint64)
    return res


def symmetry_fixtures(game_mod, n, states, seed):
    """SplendorGame.getSymmetries (SplendorGame.py:59-61 -> SplendorLogicNumba.py:349-395)
    on canonical positions with random policies; variants of position i are
    [off[i], off[i+1])."""
    g = game_mod.SplendorGame(n)
    rng = np.random.default_rng(seed)
    rec = {k: [] for k in ("src", "src_pi", "src_valids", "state", "pi", "valids")}
    off = [0]
    for st in states:
        valid = g.getValidMoves(st, 0)
        pi = (rng.random(409) * valid).astype(np.float32)
        syms = g.getSymmetries(st, pi, valid)
        rec["src"].append(st.copy())
        rec["src_pi"].append(pi)
        rec["src_valids"].append(np.asarray(valid, dtype=np.uint8))
        for s_, p_, v_ in syms:
            rec["state"].append(np.asarray(s_, dtype=np.int8).copy())
            rec["pi"].append(np.asarray(p_, dtype=np.float32))
            rec["valids"].append(np.asarray(v_, dtype=np.uint8))
        off.append(len(rec["state"]))
    res = {k: np.array(v) for k, v in rec.items()}
    res["off"] = np.array(off)
    return res


def load_arena():
    for name in ("splendor.NNet",):
        stub = types.ModuleType(name)
        stub.NNetWrapper = object            # Arena.py:10 imports it; playGames never uses it
        sys.modules[name] = stub
    _exec_module("utils", f"{REF}/utils.py")
    return _exec_module("Arena", f"{REF}/Arena.py")


def arena_fixtures(game_mod, mcts_mod, arena_mod, n, G, sims, cpuct, fpu, seed):
    """Arena.playGames (Arena.py:175-227) between two MCTS players over different hash
    networks (player 2 negates v), moves = argmax of getActionProb(temp=0, full search)
    (Coach.py:152-153). Injected draws, keyed like BatchedArena: game g deal (seed, g,
    0xFFFFFFFF), chance of ply p (seed, g, p), tie-break of player k (seed ^ (k+1), g,
    ST_BEST | p)."""
    Game = game_mod.SplendorGame
    STREAM.set_source(np.random.default_rng([seed, 1]))
    g = Game(n)
    args = _DotDict({"numMCTSSims": sims, "cpuct": cpuct, "fpu": fpu, "prob_fullMCTS": 1.0,
                     "ratio_fullMCTS": 5, "forced_playouts": False, "no_mem_optim": False,
                     "dirichletAlpha": 0.0, "temperature": [1.25, 0.8], "lag": 0})
    ctx = {"gid": -1, "ply": 0}
    acts, results = [], []
    nets = (FakeNNetC(g), FakeNNetC(g, neg=True))
    trees = [mcts_mod.MCTS(g, nets[k], args) for k in range(2)]

    def player_of(k):
        def play(x):
            ply = ctx["ply"]
            STREAM.tie = detrand.Stream(seed ^ (k + 1), ctx["gid"], ST_BEST | ply)
            a = int(np.argmax(trees[k].getActionProb(x, temp=0, force_full_search=True)[0]))
            STREAM.set_source(detrand.Stream(seed, ctx["gid"], ply))
            ctx["ply"] = ply + 1
            acts[-1].append(a)
            return a
        return play
    p1, p2 = player_of(0), player_of(1)
    arena = arena_mod.Arena(p1, p2, p2 if n == 3 else None, g, args, no_record=True)
    orig = arena.playGame

    def play_game(verbose=False, other_way=False, cur_player=None, board=None, handi=None):
        ctx["gid"] += 1
        ctx["ply"] = 0
        acts.append([])
        STREAM.set_source(detrand.Stream(seed, ctx["gid"], 0xFFFFFFFF))
        r = orig(verbose=verbose, other_way=other_way, cur_player=cur_player, board=board, handi=handi)
        results.append([float(r[0]), float(r[1]), float(r[2])])
        return r
    arena.playGame = play_game
    one, two, draws = arena.playGames(G)
    L = max(len(a) for a in acts)
    return {"one": np.array(one), "two": np.array(two), "draws": np.array(draws),
            "result": np.array(results), "plies": np.array([len(a) for a in acts]),
            "actions": np.array([a + [-1] * (L - len(a)) for a in acts], dtype=np.int16),
            "sims": np.array(sims), "cpuct": np.array(cpuct), "fpu": np.array(fpu),
            "seed": np.array(seed, dtype=np.uint64)}


def main(only=None):
    logic, numba_logic, game_mod, mcts_mod = load_reference()
    _patch_np_random()
    if only:                                 # regenerate just the named groups (round 3)
        if "nnet3" in only:
            env = np.load(os.path.join(OUT, "env_3p.npz"))
            nf = nnet_fixture(3, env["canon"][::37][:12])
            np.savez_compressed(os.path.join(OUT, "nnet_3p.npz"), **nf)
            print(f"nnet 3p: params {int(nf['n_params'])}")
        if "train" in only:
            nnet_mod = load_trainer()
            for n, dropout, seed in ((2, 0.0, 71), (2, 0.3, 72), (4, 0.0, 74)):
                env = np.load(os.path.join(OUT, f"env_{n}p.npz"))
                tf = train_fixture(nnet_mod, n, env["canon"], env["mask_canon"], E=100, bs=32, epochs=2,
                                   lr=0.001, dropout=dropout, seed=seed)
                tag = f"{n}p" + ("_dropout" if dropout else "")
                np.savez_compressed(os.path.join(OUT, f"train_{tag}.npz"), **tf)
                print(f"train {tag}: {len(tf['sample_ids'])} steps, first losses {tf['losses'][0].round(4).tolist()}")
        if "bigmcts" in only:                # round 6: configs 4 / 5 budgets
            for n, sims, seed in ((2, 1600, 6002), (4, 400, 6004)):
                bf = big_mcts_fixtures(game_mod, mcts_mod, numba_logic, n, seed, sims, n_roots=6, n_peaked=4,
                                       seq_moves=12)
                np.savez_compressed(os.path.join(OUT, f"bigmcts_{n}p.npz"), **bf)
                print(f"bigmcts {n}p: {len(bf['root'])} searches at {sims}, seq moves {len(bf['seq_root'])}")
        return
    # tables: checked by the oracle tests against its own restatement
    np.savez_compressed(
        os.path.join(OUT, "tables.npz"),
        cards1=logic.np_all_cards_1, cards2=logic.np_all_cards_2, cards3=logic.np_all_cards_3,
        nobles=logic.np_all_nobles, diff3=logic.np_different_gems_up_to_3,
        diff2=logic.np_different_gems_up_to_2, spec3=logic.np_2specs_gems_up_to_3,
        card_sym=logic.np_cards_symmetries, rsv_sym=logic.np_reserve_symmetries)
    for n, games in ((2, 10), (3, 4), (4, 4)):
        env = env_fixtures(numba_logic, n, games, seed=1000 + n)
        np.savez_compressed(os.path.join(OUT, f"env_{n}p.npz"), **env)
        end = crafted_end_cases(numba_logic, n)
        np.savez_compressed(os.path.join(OUT, f"end_{n}p.npz"), **end)
        print(f"{n}p: {len(env['state'])} states, {len(env['det_src'])} det steps, "
              f"{len(env['uniforms'])} uniforms, masks mean {env['mask_canon'].sum(1).mean():.1f}")
        fnn = fake_nn_vectors(numba_logic, n, env["canon"][::7][:40])
        np.savez_compressed(os.path.join(OUT, f"fakenn_{n}p.npz"), **fnn)
        if n in (2, 4):
            nf = nnet_fixture(n, env["canon"][::37][:12])
            np.savez_compressed(os.path.join(OUT, f"nnet_{n}p.npz"), **nf)
            print(f"nnet {n}p: params {int(nf['n_params'])}")
    cases = [(25, 1.0, 0.0, False), (100, 2.5, 0.3, False), (100, 2.5, 0.3, True),
             (25, 1.5, -0.2, False)]
    for n in (2, 4):
        mf = mcts_fixtures(game_mod, mcts_mod, numba_logic, n, seed=2000 + n, cases=cases)
        np.savez_compressed(os.path.join(OUT, f"mcts_{n}p.npz"), **mf)
        print(f"mcts {n}p: {len(mf['root'])} searches, seq moves {len(mf['seq_root'])}")
    # round 2: root noise, episodes, symmetries, arena (injected keyed draws)
    _check_legacy_choice()
    for n in (2, 3, 4):
        env = np.load(os.path.join(OUT, f"env_{n}p.npz"))
        canon = env["canon"]
        wide = wide_roots(numba_logic, n, canon[::11][:40])[:6]
        nf = noise_fixtures(game_mod, mcts_mod, numba_logic, n, list(canon[::29][:8]) + wide, seed=3000 + n)
        np.savez_compressed(os.path.join(OUT, f"noise_{n}p.npz"), **nf)
        print(f"noise {n}p: {len(nf['ps_in'])} cases, max legal {int(nf['vs'].sum(1).max())}")
        ncases = [(25, 1.5, 0.1, 0.3, 1.25, False), (60, 2.5, 0.3, 0.3, 1.25, True)]
        roots = list(canon[::41][:4]) + wide[:2]
        sf = noise_search_fixtures(game_mod, mcts_mod, n, roots, seed=3100 + n, cases=ncases)
        np.savez_compressed(os.path.join(OUT, f"noisesearch_{n}p.npz"), **sf)
        print(f"noise searches {n}p: {len(sf['root'])}")
        rsv = [st for st in canon if np.any(st[32 + 2 * n + n * (n + 1) + n:] != 0)]
        sym_states = list(canon[::23][:20]) + rsv[::max(1, len(rsv) // 20)][:20]
        yf = symmetry_fixtures(game_mod, n, sym_states, seed=3200 + n)
        np.savez_compressed(os.path.join(OUT, f"sym_{n}p.npz"), **yf)
        print(f"symmetries {n}p: {len(yf['src'])} positions, {len(yf['state'])} variants")
    coach_mod = load_coach()
    eargs = {"numMCTSSims": 24, "cpuct": 1.5, "fpu": 0.1, "prob_fullMCTS": 0.5, "ratio_fullMCTS": 4,
             "forced_playouts": False, "no_mem_optim": False, "dirichletAlpha": 0.3,
             "temperature": [1.25, 0.8], "tempThreshold": 10, "no_compression": True}
    for n, boards, forced in ((2, (3, 17), False), (2, (5,), True), (4, (2,), False)):
        a = dict(eargs, forced_playouts=forced)
        ef = episode_fixtures(game_mod, coach_mod, n, 0x5EED + n, boards, a)
        tag = f"{n}p" + ("_forced" if forced else "")
        np.savez_compressed(os.path.join(OUT, f"episode_{tag}.npz"), **ef)
        print(f"episode {tag}: moves {ef['game_moves'].tolist()}, examples {ef['game_n_examples'].tolist()}")
    arena_mod = load_arena()
    for n, G, sims in ((2, 8, 8), (3, 4, 6)):
        af = arena_fixtures(game_mod, mcts_mod, arena_mod, n, G, sims, 1.5, 0.1, seed=41 + n)
        np.savez_compressed(os.path.join(OUT, f"arena_{n}p.npz"), **af)
        print(f"arena {n}p: {int(af['one'])}-{int(af['two'])}-{int(af['draws'])}, plies {af['plies'].tolist()}")


if __name__ == "__main__":
    main(sys.argv[1].split(",") if len(sys.argv) > 1 else None)
