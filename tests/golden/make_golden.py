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
Chance injection (the reference is unseeded):
  np.random.random -> pops the next double of an injected uniform stream.
  np.random.choice(10, k, replace=False) (noble draw, SplendorLogicNumba.py:241) ->
      partial Fisher-Yates driven by the same stream: for i<k: j=i+floor(u*(10-i)).

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
import os
import sys
import types
import math

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


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

    def set_source(self, rng):
        self.src = rng
        self.used = []

    def random(self, *a, **k):
        assert not a and not k
        u = float(self.src.random())
        self.used.append(u)
        return u

    def choice(self, a, size=None, replace=True, p=None):
        assert replace is False and p is None and isinstance(a, (int, np.integer))
        perm = list(range(int(a)))
        for i in range(int(size)):
            u = self.random()
            j = i + int(math.floor(u * (int(a) - i)))
            perm[i], perm[j] = perm[j], perm[i]
        return np.array(perm[:size], dtype=np.int64)


STREAM = UniformStream()


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


def main():
    logic, numba_logic, game_mod, mcts_mod = load_reference()
    _patch_np_random()
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


if __name__ == "__main__":
    main()
