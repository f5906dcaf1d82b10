"""ctypes binding of the CPU oracle (oracle/liboracle.so). Test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "splendor_oracle.c")
        if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = C.CDLL(LIB_PATH)
        p8, pu8, pf, pd, pi = (C.POINTER(C.c_int8), C.POINTER(C.c_uint8), C.POINTER(C.c_float),
                               C.POINTER(C.c_double), C.POINTER(C.c_int))
        L.or_rows.argtypes = [C.c_int]
        L.or_init.argtypes = [C.c_int, p8, pd, pi]
        L.or_valid_moves.argtypes = [C.c_int, p8, C.c_int, pu8]
        L.or_make_move.argtypes = [C.c_int, p8, C.c_int, C.c_int, C.c_int, pd, pi]
        L.or_make_move.restype = C.c_int
        L.or_check_end.argtypes = [C.c_int, p8, pf]
        L.or_swap_players.argtypes = [C.c_int, p8, C.c_int]
        L.or_get_score.argtypes = [C.c_int, p8, C.c_int]
        L.or_get_round.argtypes = [p8]
        L.or_card.argtypes = [C.c_int, C.c_int, C.c_int, p8]
        L.or_tree_step.argtypes = [C.c_int, p8, C.c_int, p8]
        L.or_symmetries.argtypes = [C.c_int, p8, pf, pu8, p8, pf, pu8]
        L.or_uniform.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.or_uniform.restype = C.c_double
        L.or_state_hash.argtypes = [p8, C.c_int]
        L.or_state_hash.restype = C.c_uint64
        L.or_fake_predict.argtypes = [C.c_int, p8, pu8, pf, pf]
        L.or_set_fake_mode.argtypes = [C.c_int]
        L.or_depth_stats.argtypes = [C.POINTER(C.c_longlong), C.c_int]
        L.or_np_sum_f32.argtypes = [pf, C.c_int]
        L.or_np_sum_f32.restype = C.c_float
        L.or_mcts_new.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_int]
        L.or_mcts_new.restype = C.c_void_p
        L.or_mcts_free.argtypes = [C.c_void_p]
        L.or_mcts_set_net.argtypes = [C.c_void_p, C.c_int]
        L.or_mcts_set_noise.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_uint64, C.c_uint32, C.c_uint32]
        L.or_dirichlet.argtypes = [C.c_double, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, pd]
        L.or_root_noise.argtypes = [pf, pu8, pd, C.c_double]
        L.or_mcts_search.argtypes = [C.c_void_p, p8, C.POINTER(C.c_int64), pd, pd, pd]
        L.or_random_rollouts.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int]
        L.or_random_rollouts.restype = C.c_longlong
        L.or_rollout_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint32, p8, p8,
                                     C.POINTER(C.c_int16), pf, C.POINTER(C.c_int32), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64)]
        L.or_rollout_run.restype = C.c_longlong
        L.or_selfplay_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint32, C.c_int, C.c_int,
                                      C.c_double, C.c_double, C.c_double, C.c_int, C.c_int, C.c_double,
                                      C.c_double, p8,
                                      C.POINTER(C.c_int32), C.c_int, p8, pf, C.POINTER(C.c_uint64), pf,
                                      C.POINTER(C.c_int32), pf, C.POINTER(C.c_int32)]
        L.or_selfplay_run.restype = C.c_int
        L.or_philox4x32.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def rows(n):
    return lib().or_rows(n)


def init(n, uniforms):
    st = np.zeros((rows(n), 7), np.int8)
    u = np.ascontiguousarray(uniforms, np.float64)
    used = C.c_int(0)
    lib().or_init(n, _p(st, C.c_int8), _p(u, C.c_double), C.byref(used))
    return st, used.value


def valid_moves(n, state, player):
    st = np.ascontiguousarray(state, np.int8)
    m = np.zeros(409, np.uint8)
    lib().or_valid_moves(n, _p(st, C.c_int8), player, _p(m, C.c_uint8))
    return m


def make_move(n, state, action, player, deterministic, uniforms=()):
    st = np.array(state, np.int8, copy=True)
    u = np.ascontiguousarray(np.concatenate([np.asarray(uniforms, np.float64), np.zeros(4)]))
    used = C.c_int(0)
    nxt = lib().or_make_move(n, _p(st, C.c_int8), int(action), int(player), int(deterministic),
                             _p(u, C.c_double), C.byref(used))
    return st, nxt, used.value


def check_end(n, state):
    st = np.ascontiguousarray(state, np.int8)
    out = np.zeros(n, np.float32)
    lib().or_check_end(n, _p(st, C.c_int8), _p(out, C.c_float))
    return out


def swap_players(n, state, k):
    st = np.array(state, np.int8, copy=True)
    lib().or_swap_players(n, _p(st, C.c_int8), int(k))
    return st


def score(n, state, p):
    st = np.ascontiguousarray(state, np.int8)
    return lib().or_get_score(n, _p(st, C.c_int8), p)


def tree_step(n, state, action):
    st = np.ascontiguousarray(state, np.int8)
    out = np.zeros_like(st)
    nxt = lib().or_tree_step(n, _p(st, C.c_int8), int(action), _p(out, C.c_int8))
    return out, nxt


def card(tier, color, k):
    out = np.zeros((2, 7), np.int8)
    lib().or_card(tier, color, k, _p(out, C.c_int8))
    return out


def symmetries(n, state, pi, valids):
    st = np.ascontiguousarray(state, np.int8)
    pi = np.ascontiguousarray(pi, np.float32)
    va = np.ascontiguousarray(valids, np.uint8)
    mx = 1 + 9 + 2 * n
    os_ = np.zeros((mx,) + st.shape, np.int8)
    op = np.zeros((mx, 409), np.float32)
    ov = np.zeros((mx, 409), np.uint8)
    k = lib().or_symmetries(n, _p(st, C.c_int8), _p(pi, C.c_float), _p(va, C.c_uint8),
                            _p(os_, C.c_int8), _p(op, C.c_float), _p(ov, C.c_uint8))
    return os_[:k], op[:k], ov[:k]


def uniform(seed, board, stream, draw):
    return lib().or_uniform(seed, board, stream, draw)


def fake_predict(n, state, valids):
    st = np.ascontiguousarray(state, np.int8)
    va = np.ascontiguousarray(valids, np.uint8)
    pi = np.zeros(409, np.float32)
    v = np.zeros(n, np.float32)
    lib().or_fake_predict(n, _p(st, C.c_int8), _p(va, C.c_uint8), _p(pi, C.c_float), _p(v, C.c_float))
    return pi, v


def np_sum_f32(x):
    x = np.ascontiguousarray(x, np.float32)
    return np.float32(lib().or_np_sum_f32(_p(x, C.c_float), len(x)))


def dirichlet(alpha, seed, board, stream, count):
    out = np.zeros(max(count, 1), np.float64)
    lib().or_dirichlet(alpha, seed, board, stream, count, _p(out, C.c_double))
    return out[:count]


def root_noise(ps, vs, dir_values, temp0):
    """softmax(ps, temp0) -> applyDirNoise -> normalise (MCTS.py:141-144), returns float32[409]."""
    p = np.array(ps, np.float32, copy=True)
    va = np.ascontiguousarray(vs, np.uint8)
    d = np.ascontiguousarray(np.concatenate([np.asarray(dir_values, np.float64), [0.0]]))
    lib().or_root_noise(_p(p, C.c_float), _p(va, C.c_uint8), _p(d, C.c_double), float(temp0))
    return p


class Mcts:
    def __init__(self, n, sims, cpuct, fpu, forced):
        self.n = n
        self.h = lib().or_mcts_new(n, sims, cpuct, fpu, int(forced))

    def set_net(self, neg_v):
        lib().or_mcts_set_net(self.h, int(neg_v))

    def set_noise(self, alpha, temp0, seed, board, stream):
        lib().or_mcts_set_noise(self.h, alpha, temp0, seed, board, stream)

    def search(self, root):
        st = np.ascontiguousarray(root, np.int8)
        counts = np.zeros(409, np.int64)
        qsa = np.zeros(409, np.float64)
        probs = np.zeros(409, np.float64)
        q = np.zeros(self.n, np.float64)
        nodes = lib().or_mcts_search(self.h, _p(st, C.c_int8), _p(counts, C.c_int64),
                                     _p(qsa, C.c_double), _p(probs, C.c_double), _p(q, C.c_double))
        return counts, qsa, probs, q, nodes

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_mcts_free(self.h)
            self.h = None


def random_rollouts(n, B, steps, seed, threads=1):
    return lib().or_random_rollouts(n, B, steps, seed, threads)


def rollout_run(n, B, steps, seed, board_base=0, masks=False):
    """Oracle of spl_rollout_step: returns dict of final state/player and traces (with
    masks=True also every move's legality words, [steps, B, 7] uint64)."""
    S = 7 * rows(n)
    st = np.zeros((B, rows(n), 7), np.int8)
    pl = np.zeros(B, np.int8)
    act = np.zeros((steps, B), np.int16)
    end = np.zeros((steps, B, n), np.float32)
    games = np.zeros(B, np.int32)
    fold = np.zeros(B, np.uint64)
    mk = np.zeros((steps, B, 7), np.uint64) if masks else None
    lib().or_rollout_run(n, B, steps, seed, board_base, _p(st, C.c_int8), _p(pl, C.c_int8),
                         _p(act, C.c_int16), _p(end, C.c_float), _p(games, C.c_int32),
                         _p(fold, C.c_uint64), _p(mk, C.c_uint64) if masks else None)
    out = {"state": st, "player": pl, "action": act, "ended": end, "games": games, "mask_fold": fold}
    if masks:
        out["masks"] = mk
    return out


def set_fake_mode(mode):
    lib().or_set_fake_mode(int(mode))


def depth_stats(reset=True):
    """(sum, max, count) of the leaf depths of every oracle simulation since the last reset."""
    out = (C.c_longlong * 3)()
    lib().or_depth_stats(out, int(reset))
    return tuple(int(x) for x in out)


def selfplay_run(n, B, iters, seed, num_sims, ratio_full, prob_full, cpuct, fpu, forced, temp_threshold,
                 board_base=0, max_ex=20000, dir_alpha=0.0, dir_temp=1.25, fake_mode=0):
    """Oracle of the device self-play loop (spl_mcts_commit semantics). fake_mode: the hash
    network's mode (0 spread, 1 peaked); the result's "depth" = (sum, max, count) of its
    simulations' leaf depths."""
    set_fake_mode(fake_mode)
    depth_stats(reset=True)
    R = rows(n)
    board = np.zeros((B, R, 7), np.int8)
    hdr = np.zeros((B, 8), np.int32)
    st = np.zeros((max_ex, R, 7), np.int8)
    pi = np.zeros((max_ex, 409), np.float32)
    va = np.zeros((max_ex, 7), np.uint64)
    win = np.zeros((max_ex, n), np.float32)
    sd = np.zeros((max_ex, n), np.int32)
    q = np.zeros((max_ex, n), np.float32)
    meta = np.zeros((max_ex, 4), np.int32)
    k = lib().or_selfplay_run(n, B, iters, seed, board_base, num_sims, ratio_full, prob_full, cpuct, fpu,
                              int(forced), temp_threshold, dir_alpha, dir_temp, _p(board, C.c_int8), _p(hdr, C.c_int32), max_ex,
                              _p(st, C.c_int8), _p(pi, C.c_float), _p(va, C.c_uint64), _p(win, C.c_float),
                              _p(sd, C.c_int32), _p(q, C.c_float), _p(meta, C.c_int32))
    k = min(k, max_ex)
    depth = depth_stats(reset=True)
    set_fake_mode(0)
    return {"board": board, "hdr": hdr, "ex_board": st[:k], "pi": pi[:k], "valids": va[:k],
            "winner": win[:k], "scdiff": sd[:k], "surprise": q[:k], "meta": meta[:k], "depth": depth}


ST_FULL, ST_DIR, ST_PICK, ST_MOVE, ST_DEAL, ST_BEST = (1 << 24), (2 << 24), (3 << 24), (4 << 24), (5 << 24), (6 << 24)
DEAL_DRAWS = 29


def one_vs_two(i):
    """Arena.py:199: player 1 moves first in games i % 4 in (0, 3)."""
    return (i % 4 == 0) or (i % 4 == 3)


def arena_play(n, G, sims, cpuct, fpu, seed, neg2=False):
    """Sequential restatement of Arena.playGames (Arena.py:64-227) on the oracle: per game
    two persistent trees (reset between games), temp-0 moves = the best root count with the
    Philox tie-break (seed ^ (k+1), game, ST_BEST | ply), chance (seed, game, ply), deal
    (seed, game, 0xFFFFFFFF); seats [p1] + [p2] * (n - 1) or the mirror. Player 2's network
    negates values when neg2. Returns per game (result vector, plies, scores, actions)."""
    out = []
    for gid in range(G):
        st, _ = init(n, [uniform(seed, gid, 0xFFFFFFFF, k) for k in range(DEAL_DRAWS)])
        seats = [0] + [1] * (n - 1) if one_vs_two(gid) else [1] + [0] * (n - 1)
        trees = [Mcts(n, sims, cpuct, fpu, False) for _ in range(2)]
        if neg2:
            trees[1].set_net(1)
        result, plies, actions = np.zeros(n, np.float32), 0, []
        for ply in range(62 * n * 2 + 8):
            cur = ply % n
            canon = swap_players(n, st, cur) if cur else st.copy()
            k = seats[cur]
            counts = trees[k].search(canon)[0]
            u = uniform(seed ^ (k + 1), gid, ST_BEST | ply, 0)
            top = counts.max()
            if top == 0:
                a = int(u * 409)
            else:
                best = np.flatnonzero(counts == top)
                a = int(best[int(u * len(best))])
            assert valid_moves(n, canon, 0)[a]
            actions.append(a)
            st, _, _ = make_move(n, st, a, cur, False, [uniform(seed, gid, ply, d) for d in range(8)])
            r = check_end(n, st)
            if r.any():
                result, plies = r, ply + 1
                break
        out.append((result, plies, [score(n, st, p) for p in range(n)], actions))
    return out


def _selfplay_part(a):
    args, kw = a
    return selfplay_run(*args, **kw)


def selfplay_run_parallel(n, B, iters, seed, num_sims, ratio_full, prob_full, cpuct, fpu, forced, temp_threshold,
                          lag=None, workers=None, **kw):
    """selfplay_run over board ids 0 .. B-1 split into contiguous parts run in worker
    processes (every draw is keyed by the global board id, so parts are independent; the
    oracle's depth statistics are per process). Board t runs iters - lag[t] iterations (a
    device tree that withdrew w simulations is exactly w simulations behind). Returns the
    concatenated result; "depth" = (sum, max, count) over all parts."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import os
    lag = np.zeros(B, np.int64) if lag is None else np.asarray(lag, np.int64)
    if workers is None:
        try:
            workers = len(os.sched_getaffinity(0))
        except AttributeError:
            workers = os.cpu_count() or 1
        workers = max(1, min(16, workers))
    size = max(1, -(-B // workers))
    parts, t0 = [], 0
    while t0 < B:
        t1 = t0 + 1
        while t1 < B and t1 - t0 < size and lag[t1] == lag[t0]:
            t1 += 1
        parts.append(((n, t1 - t0, iters - int(lag[t0]), seed, num_sims, ratio_full, prob_full, cpuct, fpu, forced,
                       temp_threshold), dict(kw, board_base=kw.get("board_base", 0) + t0)))
        t0 = t1
    with cf.ProcessPoolExecutor(max_workers=min(workers, len(parts)), mp_context=mp.get_context("spawn")) as ex:
        res = list(ex.map(_selfplay_part, parts))
    out = {k: np.concatenate([r[k] for r in res]) for k in res[0] if k != "depth"}
    d = [r["depth"] for r in res]
    out["depth"] = (sum(x[0] for x in d), max(x[1] for x in d), sum(x[2] for x in d))
    return out
