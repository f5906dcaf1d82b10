#!/usr/bin/env python3
"""Benchmark of the MI355X Splendor self-play hot path (BASELINE.json).

Headline = BASELINE.json's metric, "self-play rollouts/sec (32k boards, 2p Splendor)", a
rollout being one MCTS simulation (BASELINE.md units): BASELINE config 3, 32,768 concurrent
self-play games per GPU, numMCTSSims=100 with genbu.pt's search arguments, SplendorNNet leaf
evaluation by the fused fp32 MFMA kernel (random init: genbu.pt cannot be loaded safely),
moves, examples and re-rooting on device. One bench "step" = one self-play iteration: one
simulation (select -> network -> expand/backup) on every game plus the move commit of every
game whose search is done. The games are first brought to a steady state (--prefill
iterations: games at every stage, trees at their steady size — the synthetic input), then W
warm-up steps, then exactly K timed steps; after them an extended window (--window
iterations, default ~68 K finished games) reports capacity events, finished examples drained
+ gathered, and tree sizes.

Secondary objects in the same line (N = 1 only): config 2 (env-step-only random policy,
fused rollout kernel, board-steps/s), config 5 (4 players, 16,384 games, 400 simulations)
and config 4's per-GPU shard (32,768 games, 1,600 simulations), each at steady state with
its window statistics and CPU baselines (the oracle, a scalar C port of the reference, on
one host core and on every granted core).

Contract: `python bench.py --gpus N --steps K --warmup W`; for N>1 one rank per GPU, either
launched by torch.distributed.run (WORLD_SIZE set: it must equal N) or, when started
directly, by bench.py itself (a child torch.distributed.run of N ranks, started before
anything touches the GPU); games are sharded by board id (board_base = rank * B), examples
all-gathered over RCCL at the end of the window; rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))

import torch  # noqa: E402

METRIC = "self-play rollouts/sec (32k boards, 2p Splendor) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP32_MFMA_PEAK = 157.3    # TFLOP/s, dense fp32 MFMA (MI355X_MICROARCH.md)
BF16_MFMA_PEAK = 2500.0   # TFLOP/s, dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
RAMP_S = 0.05             # untimed launches before the env window (GPU clock ramp)
_T0 = time.perf_counter()


def log(msg):
    """Progress on stderr (a long run keeps writing, so it is never taken for a hang)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def bytes_per_board_step(n):
    """SURVEY.md §8(d) algorithmic bytes of one board-step: state read + write (2S), packed
    mask (52 = ceil(409/8)), action (2), end result (4n): 846 B for 2 players."""
    S = 7 * (32 + 10 * n + n * n)
    return 2 * S + 52 + 2 + 4 * n


def bytes_per_board_launch(n, moves):
    """Bytes one rollout launch actually moves across HBM per board: boards
    stay on chip for the launch, so state read + write (2S), player (2) and game counter (8)
    once, and per move the packed mask (56), action (2) and end result (4n)."""
    S = 7 * (32 + 10 * n + n * n)
    return 2 * S + 2 + 8 + moves * (56 + 2 + 4 * n)


def _oracle_lib():
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    L = ctypes.CDLL(path)
    L.or_random_rollouts.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
    L.or_random_rollouts.restype = ctypes.c_longlong
    return L


def host_threads():
    """Host cores this process may use (the GPU box grants a 16-core share of a larger
    machine; os.cpu_count() reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(n, seed, target_s=5.0):
    """Time the oracle (scalar C port of the reference rules, oracle/) on a bounded sample of
    the same workload (same boards, same Philox draws): one host core (the reference's
    Numba path is single-threaded) and every granted core (boards split across threads).
    `value` is the all-core rate."""
    L = _oracle_lib()
    B = 32768

    def timed(threads):
        t = time.perf_counter()
        L.or_random_rollouts(n, B, 2, seed, threads)
        probe = time.perf_counter() - t
        steps = max(2, int(target_s / max(probe / 2, 1e-6)))
        t = time.perf_counter()
        done = L.or_random_rollouts(n, B, steps, seed, threads)
        return done, steps, time.perf_counter() - t

    log("cpu baseline: rollouts")
    d1, s1, t1 = timed(1)
    T = host_threads()
    dT, sT, tT = timed(T)
    return {"value": dT / tT, "unit": "rollouts/s", "cores": T, "kind": "port",
            "sample": f"{B} boards x {sT} steps (incl. initial deal) on {T} host threads, {tT:.1f} s, "
                      f"oracle/splendor_oracle.c or_random_rollouts",
            "single_core": {"value": d1 / t1, "cores": 1,
                            "sample": f"{B} boards x {s1} steps on 1 host core, {t1:.1f} s"}}


def _selfplay_cpu_worker(args):
    """One host core: the oracle's self-play search on its own 8 games (board ids shifted by
    its index) for `iters` iterations, then `k` batch-1 SplendorNNet CPU forwards (PyTorch
    fp32, one intra-op thread) — both timed."""
    n, seed, sims, iters, k, i = args
    import numpy as np
    torch.set_num_threads(1)
    L = _oracle_lib()
    p8, pf = ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(ctypes.c_float)
    L.or_selfplay_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, p8,
                                  ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                  p8, pf, ctypes.POINTER(ctypes.c_uint64), pf, ctypes.POINTER(ctypes.c_int32), pf,
                                  ctypes.POINTER(ctypes.c_int32)]
    L.or_selfplay_run.restype = ctypes.c_int
    R = 32 + 10 * n + n * n
    g = dict(GENBU_ARGS, numMCTSSims=sims)
    B = 8
    board = np.zeros((B, R, 7), np.int8)
    hdr = np.zeros((B, 8), np.int32)

    def search(it):
        t = time.perf_counter()
        L.or_selfplay_run(n, B, it, seed, B * i, g["numMCTSSims"], g["ratio_fullMCTS"], g["prob_fullMCTS"],
                          g["cpuct"], g["fpu"], int(g["forced_playouts"]), g["tempThreshold"],
                          g["dirichletAlpha"], g["temperature"][0], board.ctypes.data_as(p8),
                          hdr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 0,
                          None, None, None, None, None, None, None)
        return time.perf_counter() - t
    from splendor.nnet import random_net
    net = random_net(n, seed=0, device="cpu")
    x = torch.zeros((1, R, 7))
    va = torch.ones((1, 409), dtype=torch.bool)
    with torch.no_grad():
        for _ in range(20):
            net(x, va)
        if iters is None:                                # probe: size the sample
            return search(10)
        dt = search(iters)
        t = time.perf_counter()
        for _ in range(k):
            net(x, va)
        nn = (time.perf_counter() - t) / k
    return B * iters / dt, nn, dt


def cpu_baseline_selfplay(n, seed, sims, target_s=4.0):
    """CPU reference point for the self-play configs (rollouts = MCTS simulations): the
    oracle's sequential search + self-play loop (oracle/splendor_oracle.c or_selfplay_run,
    hash-prior network, genbu search args) timed directly, plus one SplendorNNet forward at
    batch 1 on the CPU per simulation (PyTorch fp32, as GenericNNetWrapper.predict does per
    leaf) timed separately: per core, value = 1 / (1/search + network). On one host core (the
    reference's self-play is single-threaded) and on every granted core: T worker processes
    (one core each, their own games) run at once and their rates add up."""
    import multiprocessing as mp
    log(f"cpu baseline: {n} players, {sims} sims")
    ctx = mp.get_context("spawn")
    T = host_threads()
    with ctx.Pool(1) as pool:
        probe = pool.map(_selfplay_cpu_worker, [(n, seed, sims, None, 0, 0)])[0]
        iters = max(10, int(10 * target_s / 2 / max(probe, 1e-6)))
        r1, nn1, dt1 = pool.map(_selfplay_cpu_worker, [(n, seed, sims, iters, 200, 0)])[0]
    with ctx.Pool(T) as pool:
        res = pool.map(_selfplay_cpu_worker, [(n, seed, sims, iters, 200, i) for i in range(T)])
    one = 1.0 / (1.0 / r1 + nn1)
    allc = sum(1.0 / (1.0 / r + nnv) for r, nnv, _ in res)
    dts = max(d for _, _, d in res)
    nnT = sum(v for _, v, _ in res) / T
    return {"value": allc, "unit": "rollouts/s (MCTS simulations)", "cores": T, "kind": "port",
            "sample": f"{T} processes (one core each) x oracle self-play 8 games x {iters} simulations ({dts:.1f} s) "
                      f"+ SplendorNNet batch-1 CPU forward, {nnT * 1e6:.0f} us per leaf (PyTorch fp32, 1 thread), "
                      f"all at once; value = sum over processes of 1 / (1/search + network)",
            "single_core": {"value": one, "cores": 1,
                            "sample": f"8 games x {iters} simulations ({dt1:.1f} s, search alone {r1:.0f} sims/s) + "
                                      f"{nn1 * 1e6:.0f} us network per leaf"},
            "network_us_per_leaf": nnT * 1e6}


# saved args of the reference's only checkpoint, genbu.pt, = BASELINE config 3
GENBU_ARGS = dict(numMCTSSims=100, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5,
                  forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)


def nn_flops_per_eval(n):
    """SplendorNNet inference FLOPs per leaf (2 x MACs; score-diff head skipped)."""
    R = 32 + 10 * n + n * n
    macs = 7 * (R * 128 + 128 * 128) + 7 * 96 * 120 + 7 * 128 * 128 + 704 * 128 + 112 * 120 \
        + 2 * 128 * 128 + 112 * 120 + 128 * 128 + 128 * 409 + 128 * 128 + 128 * n
    return 2 * macs


def nn_mfma_per_tile(n):
    """MFMA instructions k_nn_forward issues per 32-leaf tile (csrc/nnet.hip): the 4 per-column
    layers on v_mfma_f32_32x32x16_bf16 (7 token tiles x 4 column tiles; three part products
    per 16-k chunk for dense2d_1's exact int8 input, six for the others) and the 9 per-leaf
    layers on v_mfma_f32_16x16x32_bf16 (2 row tiles x the column tiles; six per 32-k chunk),
    K rounded up to the chunk and N to the tile as the kernel runs them."""
    R = 32 + 10 * n + n * n
    c16 = lambda K: (K + 15) // 16
    c32 = lambda K: (K + 31) // 32
    t16 = lambda N: (N + 15) // 16
    m32 = 28 * (3 * c16(R) + 6 * (c16(128) + c16(96) + c16(128)))
    leaf = [(128, 704), (120, 112), (128, 128), (128, 128), (120, 112), (128, 128), (409, 128), (128, 128), (n, 128)]
    m16 = sum(2 * t16(N) * c32(K) * 6 for N, K in leaf)
    return m32, m16


def nn_mix_ceiling_us(n, leaves):
    """The MFMA floor of the shipping instruction mix: the bf16 MFMA FLOPs k_nn_forward
    executes over `leaves` leaves (whole 32-leaf tiles) at the dense bf16 peak."""
    m32, m16 = nn_mfma_per_tile(n)
    flops = ((leaves + 31) // 32) * (m32 * 32 * 32 * 16 * 2 + m16 * 16 * 16 * 32 * 2)
    return flops / (BF16_MFMA_PEAK * 1e12) * 1e6, flops


def bytes_per_rollout(n, depth):
    """SURVEY.md §8(d) algorithmic HBM bytes of one MCTS simulation: leaf state as the f32
    network input (4S), bool mask (409), f32 policy out (4 x 409), f32 values (4n), and the
    path (16 B per level: P, Q, N, child). §8(d) uses the reference's measured depth 4.8
    (3.7 KB at 2 players); `depth` = the measured mean leaf depth of the trees here."""
    S = 7 * (32 + 10 * n + n * n)
    return 4 * S + 409 + 4 * 409 + 4 * n + 16 * depth


CONFIGS = {  # BASELINE.json configs: (players, games per GPU, numMCTSSims)
    "config3": (2, 32768, 100),
    "config4": (2, 32768, 1600),
    "config5": (4, 16384, 400),
}
# per workload: untimed prefill iterations to the steady state, the phase stagger inside it
# (~ one game length), and the statistics window after the timed steps
PHASES = {
    "config3": dict(prefill=6000, stagger=4800, window=10000),
    # config 4: a game is ~76 K iterations (0.25 x 1,600 + 0.75 x 320 simulations per move, ~119
    # plies), so the stagger spans one game (restarts every 4,800 iterations) and the prefill
    # ends with the games' ages spread over 12 K .. 84 K iterations (45 K / 40 K had
    # left the window with 39 finished games, i.e. no end-game phases)
    "config4": dict(prefill=84000, stagger=80000, window=4000),
    "config5": dict(prefill=40000, stagger=32000, window=6000),
}


def stagger_marks(stagger, groups, sims, ratio):
    """(iteration, group) restart points of run_selfplay's phase stagger: group j restarts
    after j * step iterations, step = stagger / groups rounded down to a multiple of the
    fast-search budget sims // ratio (so the restarted games keep the search boundaries
    every game dealt at iteration 0 has); none when the stagger is shorter than that."""
    fast = max(1, sims // ratio)
    step = stagger // groups // fast * fast
    return [(j * step, j) for j in range(1, groups)] if step else []


def run_selfplay(cfg, rank, world, dev, dist, steps, warmup, prefill, window, seed, node_boards=-1,
                 stagger=0, groups=16, mem_gib=0.0, on_steady=None, net_path=None):
    """Self-play at one BASELINE config: B games per GPU (shard board_base = rank * B), one
    MCTS simulation per game per iteration, leaves evaluated by the fused SplendorNNet kernel
    (fp32, random init), moves committed on device. `prefill` untimed iterations bring the
    games to a steady state, `warmup` more, then exactly `steps` timed iterations (barrier +
    synchronize on both sides, max over ranks); then `window` iterations whose statistics
    (capacity events, games, moves) are reported, ending with the finished examples drained
    and all-gathered over RCCL; symmetry expansion is timed after it.

    stagger: the B games are dealt together, so without it they share one game phase for
    many generations and the per-iteration cost oscillates with it (config 3: 0.56-0.95 ms
    over a ~4,800-iteration period: end-game trees reach terminal states, which need no
    network evaluation). Within the prefill, group j of `groups` (trees t % groups == j)
    abandons its game and is dealt a new one after j * (stagger // groups) iterations, so the
    games' phases end up spread over `stagger` iterations (~ one mean game length): the
    population a long-running self-play reaches, every phase equally represented. The
    restarts fall on multiples of the fast-search budget (numMCTSSims / ratio_fullMCTS): with
    one simulation per tree per iteration, games dealt together keep their search boundaries
    aligned for good (every search spends 100 or 20 simulations, so all of them end in the
    same iterations, one in 20), and so do the restarted ones, as a self-play run whose games
    were all dealt at once does. (Restarts off that grid spread the boundaries over all
    iterations: config 3 then runs ~14 % slower, since every select launch then carries some
    deep descents.)"""
    from splendor.coach import expand_symmetries
    from splendor.env import SplendorEngine
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.selfplay import SelfPlay, broadcast_network, gather_examples
    n, B, sims = CONFIGS[cfg]
    eng = SplendorEngine(n, device=dev)
    sargs = dict(GENBU_ARGS, numMCTSSims=sims)
    net = random_net(n, seed=rank, device=dev)
    if net_path:                               # trained weights (tools/train_prior.py): a plain
        data = torch.load(net_path, map_location=dev, weights_only=True)      # state_dict only
        net.load_state_dict(data["state_dict"] if "state_dict" in data else data)
        net.eval()
    if dist:
        broadcast_network(net)                 # every rank searches with rank 0's network
    ev = LeafEvaluator(eng, net, B, use_graph=False)
    sp = SelfPlay(eng, B, sargs, evaluator=ev, dirichlet_noise=True, seed=seed, board_base=rank * B,
                  node_boards=None if node_boards < 0 else bool(node_boards),
                  mem_budget=int(mem_gib * 2**30) if mem_gib > 0 else None)
    sp.reset()
    t_fill = time.perf_counter()
    done = 0
    log(f"{cfg}: {B} games, {sims} sims, pools {sp.cfg.pool_nodes} nodes / {sp.cfg.pool_edges} edges, "
        f"node boards {sp.cfg.node_boards}, {sp.device_bytes / 2**30:.1f} GiB; prefill {prefill}")
    stagger = min(stagger, prefill)
    marks = stagger_marks(stagger, groups, sims, GENBU_ARGS["ratio_fullMCTS"])
    for target, j in marks + [(prefill, None)]:
        while done < target:                   # (in chunks: a sync now and then keeps the
            k = min(2000, target - done)       #  host's view of progress; drained as it goes)
            sp.run(k, use_graph=True)
            done += k
            sp.drain(allow_drops=False)
            torch.cuda.synchronize(dev)
            log(f"{cfg}: prefill {done}/{prefill}")
        if j is not None:                      # group j starts a new game (phase spreading)
            sp.restart(torch.arange(B) % groups == j)
    prefill_s = time.perf_counter() - t_fill
    sp.run(max(warmup, 1), use_graph=True)
    sp.drain()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ev1.record()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if on_steady:
        on_steady(sp)                          # (diagnostic tools: counters reset here)
    t0 = time.perf_counter()
    ev0.record()
    sp.run(steps, use_graph=True)
    ev1.record()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    iter_ms_events = ev0.elapsed_time(ev1) / steps
    # extended window: capacity events, games, examples drained + gathered
    c0 = sp.counter_snapshot()
    pool0 = sp.pool_state()
    ex_local = 0
    tw = time.perf_counter()
    done = 0
    log(f"{cfg}: timed {steps} iterations, {elapsed:.2f} s; window {window}")
    while done < window:
        k = min(2000, window - done)
        sp.run(k, use_graph=True)
        done += k
        if done < window:
            ex_local += int(sp.drain()["board"].shape[0])
            log(f"{cfg}: window {done}/{window}")
    torch.cuda.synchronize(dev)
    tg = time.perf_counter()
    ex = sp.drain()
    ex_local += int(ex["board"].shape[0])
    if dist:
        ex = gather_examples(ex)
    torch.cuda.synchronize(dev)
    gather_s = time.perf_counter() - tg
    window_s = time.perf_counter() - tw
    st = sp.stats()
    pool = sp.pool_state()
    ts = sp.tree_sizes()
    # the share of simulations whose leaf needs the network (the rest end on a terminal
    # state): the compacted NN-leaf count of 200 single iterations
    nn_leaves = 0
    for _ in range(200):
        sp.run(1, use_graph=True)
        nn_leaves += int(sp.leaf_count.sum().item())
    nn_leaf_frac = nn_leaves / (200 * B)
    nsym = min(int(ex["board"].shape[0]), 200000)
    t_s = time.perf_counter()
    sym = expand_symmetries(eng, {k: v[:nsym] for k, v in ex.items()}) if nsym else None
    torch.cuda.synchronize(dev)
    sym_s = time.perf_counter() - t_s
    # the network kernel on its own: k_nn_forward over B leaves, HIP events on its stream
    nk = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(10):
        ev(sp.leaf_state, sp.leaf_mask)
    e0.record()
    for _ in range(nk):
        ev(sp.leaf_state, sp.leaf_mask)
    e1.record()
    torch.cuda.synchronize(dev)
    nn_us = e0.elapsed_time(e1) / nk * 1e3
    delta = sp.counter_delta(c0, sp.counter_snapshot())     # per tree, modulo 2^32, then summed
    # leaf depth over every simulation backed up in the window (a snapshot of the trees'
    # current path depths swings with the 20-iteration search cycle)
    depth_mean = delta["depth_sum"] / delta["sims_backed"] if delta["sims_backed"] else st["leaf_depth_now"]
    delta["iterations"] = window
    delta["seconds"] = window_s
    delta["rollouts_per_s"] = world * B * window / window_s
    delta["node_page_misses"] = pool["node_page_misses"] - pool0["node_page_misses"]
    delta["edge_page_misses"] = pool["edge_page_misses"] - pool0["edge_page_misses"]
    # steady-state check: at a steady population every game finishes within the window at the
    # rate B / (game length), i.e. the window's moves per finished game ~ plies per game (~119 at
    # 2 players); a population still in its first games shows thousands
    delta["moves_per_game_finished"] = delta["moves"] / max(1, delta["games_done"])
    delta["events_per_1000_moves"] = {k: 1000.0 * delta[k] / max(1, delta["moves"])
                                      for k in ("prunes", "resets", "unexpanded")}
    delta["examples_drained"] = ex_local
    delta["examples_gathered"] = int(ex["board"].shape[0])
    if dist:
        t = torch.tensor([ex_local], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        delta["examples_drained_all_ranks"] = int(t.item())
    delta["drain_allgather_s"] = gather_s
    live_n, live_e = ts[:, 2].astype("int64"), ts[:, 3].astype("int64")
    tree = {"nodes_max": st["nodes_max"], "edges_max": st["edges_max"],
            "live_nodes_mean": float(live_n.mean()), "live_nodes_max": int(live_n.max()),
            "live_edges_mean": float(live_e.mean()), "live_edges_max": int(live_e.max()),
            "leaf_depth_mean": depth_mean, "leaf_depth_max": st["depth_max_all"],
            "leaf_depth_mean_note": "window depth_sum / simulations backed up (every simulation's leaf depth)",
            "overflow": st["overflow"], "examples_dropped": st["examples_dropped"],
            "node_cap_per_tree": int(sp.cfg.node_cap), "pool_nodes": int(sp.cfg.pool_nodes),
            "pool_edges": int(sp.cfg.pool_edges), "node_boards": int(sp.cfg.node_boards),
            "device_bytes": sp.device_bytes,
            "pool_free_at_end": {"node_pages": pool["free_node_pages"], "of": pool["node_pages"],
                                 "edge_pages": pool["free_edge_pages"], "of_edge": pool["edge_pages"]}}
    res = {"elapsed": elapsed, "iter_ms_events": iter_ms_events, "window": delta, "tree": tree,
           "prefill": prefill, "prefill_s": prefill_s, "stagger": {"iterations": stagger, "groups": groups},
           "symmetry": {"examples": nsym, "variants": int(sym["board"].shape[0]) if sym else 0, "s": sym_s},
           "nn_kernel_us": nn_us, "nn_leaf_fraction": nn_leaf_frac}
    del sp, ev, net
    return res


def selfplay_record(cfg, r, world, steps, warmup):
    """The JSON object of one self-play config."""
    n, B, sims = CONFIGS[cfg]
    fl = nn_flops_per_eval(n) * B
    return {"workload": f"{cfg}: {n}-player batched self-play, {B} games per GPU, numMCTSSims={sims}, genbu "
                        "search args, SplendorNNet fp32 leaf eval (random init), device move commit",
            "value": world * B * steps / r["elapsed"], "unit": "rollouts/s (MCTS simulations)",
            "n_gpus": world, "global_games": world * B,
            "ms_per_iteration": r["elapsed"] / steps * 1e3, "ms_per_iteration_events": r["iter_ms_events"],
            "steps": steps, "warmup": warmup, "prefill_iterations": r["prefill"], "prefill_s": r["prefill_s"],
            "phase_stagger": r["stagger"],
            "window": r["window"], "tree": r["tree"], "symmetry_expansion": r["symmetry"],
            # every search ran on the reference's table (no prune / reset / unexpanded leaf in the
            # window; withdrawals repeat a simulation exactly): False marks a non-conforming record
            "reference_table": not any(r["window"].get(k, 0) for k in ("prunes", "resets", "unexpanded")),
            "nn_leaf_fraction": r["nn_leaf_fraction"],
            "network_kernel": _network_kernel(n, B, r["nn_kernel_us"])}


def _network_kernel(n, B, us):
    """k_nn_forward alone over B leaves: f32-equivalent throughput (the network's FLOPs) and
    the bf16 MFMA throughput it executes (six part products per f32 product), the latter
    against the dense bf16 peak and the instruction mix's MFMA floor."""
    fl = nn_flops_per_eval(n) * B
    ceil_us, xfl = nn_mix_ceiling_us(n, B)
    return {"kernel": f"k_nn_forward<{n}>", "avg_us": us,
            "tflops_f32_equivalent": fl / (us * 1e-6) / 1e12,
            "frac_fp32_mfma_peak": fl / (us * 1e-6) / 1e12 / FP32_MFMA_PEAK,
            "executed_bf16_tflops": xfl / (us * 1e-6) / 1e12,
            "frac_bf16_mfma_peak": xfl / (us * 1e-6) / 1e12 / BF16_MFMA_PEAK,
            "executed_bf16_flop_per_launch": xfl, "mix_ceiling_us": ceil_us, "frac_of_mix_ceiling": ceil_us / us,
            "note": "k_nn_forward alone over B leaves (HIP events, 10 warm-up + 50 timed launches); f32 "
                    "arithmetic as bf16 part products: 'f32-equivalent' counts the network's own FLOPs "
                    "(1.19 MFLOP per leaf), 'executed' the bf16 MFMA FLOPs issued"}


def load_json_profile(pattern):
    """The newest committed summary matching profiles/<pattern> (sorted names: rNN order)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not paths:
        return None
    with open(paths[-1]) as f:
        return dict(json.load(f), file=os.path.relpath(paths[-1], ROOT))


def load_traffic(path, B, moves):
    """The newest committed rocprofv3 --pmc summary of the rollout workload (profiles/
    rNN_rollout_pmc*.json, tools/pmc_rollout.sh; HBM bytes corrected as DESIGN.md §5
    describes), if it was taken at this board count and launch size."""
    import glob
    paths = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_rollout_pmc*.json")))
    best = None
    for p in paths:
        if not os.path.exists(p):
            continue
        with open(p) as f:
            d = json.load(f)
        if d.get("boards") == B and d.get("moves_per_launch", 1) == moves:
            best = dict(d, file=os.path.relpath(p, ROOT))        # newest round wins (sorted names)
    return best


def selfplay_roofline(rec, n, depth):
    """Roofline block of the headline: the dominant kernel is k_nn_forward (MFMA-bound, f32
    arithmetic; per-column layers on split-bf16 MFMAs, see mfma_mix):
    achieved = 1.19 MFLOP per leaf x B leaves / its HIP-event launch time. traffic = its HBM
    bytes per launch from the newest committed PMC summary (profiles/rNN_selfplay_pmc.json,
    tools/pmc_selfplay.sh); the tree kernels' measured bytes per simulation are set beside
    SURVEY §8(d)'s algorithmic figure."""
    nk = rec["network_kernel"]
    prof = load_json_profile("r*_selfplay_pmc.json")
    kern = (prof or {}).get("kernels", {})
    B = CONFIGS["config3"][1]
    # the network kernel over the same full batch under rocprofv3 (duration, PMC bytes):
    # profiles/rNN_nn_fullbatch.json (tools/nn_fullbatch.sh); the self-play PMC summary's
    # k_nn_forward entry covers the compacted launches (~72 % of the leaves) instead
    nnfb = load_json_profile("r*_nn_fullbatch.json") or {}

    def per_sim(k):
        v = kern.get(k, {}).get("hbm_bytes_per_launch")
        return v / B if v else None
    tree = {k: {"hbm_bytes_per_sim": per_sim(k), "avg_us_rocprof": kern.get(k, {}).get("avg_us")}
            for k in ("k_select", "k_backup", "k_leaf_mask", "k_commit", "k_gc")}
    tot = sum(v["hbm_bytes_per_sim"] or 0.0 for v in tree.values())
    return {"bound": "mfma", "achieved": nk["executed_bf16_tflops"], "peak": BF16_MFMA_PEAK, "unit": "TFLOP/s",
            "frac": nk["frac_bf16_mfma_peak"],
            "mfma_mix": "f32 arithmetic (the reference's precision) with every f32 operand split exactly into "
                        "three bf16 parts: the 4 per-column layers on v_mfma_f32_32x32x16_bf16, the 9 per-leaf "
                        "layers on v_mfma_f32_16x16x32_bf16 (six part products per chunk, DESIGN.md §4); "
                        "achieved = the bf16 MFMA FLOPs executed, against the dense bf16 peak",
            "mix_ceiling_us": nk["mix_ceiling_us"], "frac_of_mix_ceiling": nk["frac_of_mix_ceiling"],
            "f32_equivalent": {"achieved": nk["tflops_f32_equivalent"], "peak": FP32_MFMA_PEAK,
                               "frac": nk["frac_fp32_mfma_peak"],
                               "note": "the network's own f32 FLOPs per second against the f32 MFMA peak: an "
                                       "f32-equivalent throughput, not the utilisation of the pipe that runs "
                                       "them (may exceed 1)"},
            "traffic": nnfb.get("hbm_bytes_per_launch"),
            "kernel": nk["kernel"], "kernel_avg_us": nk["avg_us"],
            "kernel_avg_us_rocprof": nnfb.get("avg_us"), "rocprof_file": nnfb.get("file"),
            "selfplay_launch": {"avg_us_rocprof": kern.get("k_nn_forward", {}).get("avg_us"),
                                "hbm_bytes_per_launch": kern.get("k_nn_forward", {}).get("hbm_bytes_per_launch"),
                                "note": "in self-play the kernel runs on the compacted NN-leaf list"},
            "flop_per_launch": nn_flops_per_eval(n) * B,
            "tree_kernels": {"per_kernel": tree, "hbm_bytes_per_sim_total": tot or None,
                             "algorithmic_bytes_per_sim_survey": bytes_per_rollout(n, 4.8),
                             "algorithmic_bytes_per_sim_at_measured_depth": bytes_per_rollout(n, depth),
                             "note": "PMC FETCH_SIZE x1024 x2 (gfx950) + WRITE_SIZE x1024 per launch / B"},
            "pmc_file": (prof or {}).get("file")}


def run_env(args, rank, world, dev, dist, K, warmup, cpu=True):
    """BASELINE config 2: 32,768 boards, uniform-random legal actions, fused rollout kernel
    (canonical form -> mask -> action -> chance step -> end check -> auto-reset), K moves in
    launches of --chunk moves, HIP events on the launch stream around the timed launches."""
    from splendor.env import RolloutBatch, SplendorEngine
    eng = SplendorEngine(args.players if args.workload == "env" else 2, device=dev)
    n = eng.n
    B = args.boards
    rb = RolloutBatch(eng, B, seed=args.seed, board_base=rank * B)
    chunk = max(1, min(args.chunk, K))
    launches = [chunk] * (K // chunk) + ([K % chunk] if K % chunk else [])
    outs = {}

    def run(k):
        outs[k] = rb.run(k, out=outs.get(k))
    w = warmup
    while w > 0:
        run(min(chunk, w))
        w -= chunk
    for k in set(launches):
        run(k)                                 # output buffers of every launch size exist
    launchers = {k: rb.launcher(k, outs[k]) for k in set(launches)}
    # clock ramp: an idle GPU starts the timed launches at a low clock; untimed launches of
    # the timed size for ~RAMP_S seconds first (the boards just play on)
    ramp = 0
    t_r = time.perf_counter()
    while time.perf_counter() - t_r < RAMP_S:
        launchers[chunk]()
        ramp += 1
        if ramp % 16 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ev1.record()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    seq = [launchers[k] for k in launches]
    t0 = time.perf_counter()
    ev0.record()
    for fn in seq:
        fn()
    ev1.record()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = ev0.elapsed_time(ev1) / len(launches)
    games = int(rb.games.sum().item())
    del rb, outs, launchers
    torch.cuda.empty_cache()
    step_b = bytes_per_board_step(n)
    achieved = step_b * B * chunk / (kernel_ms * 1e-3) / 1e9
    moved = bytes_per_board_launch(n, chunk)
    moved_gbs = moved * B / (kernel_ms * 1e-3) / 1e9
    prof = load_traffic(args.traffic_json, B, chunk)
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    issue = ({k: prof.get(k) for k in ("valu_insts_per_board_move", "valu_issue_frac", "effective_clock_ghz",
                                        "kernel_avg_us_rocprof", "file")}
             if prof else None)
    rec = {"workload": "config2: env-step-only random-policy self-play, fused canonical+mask+action+chance "
                       "step+end check+auto-reset",
           "value": world * B * K / elapsed, "unit": "board-steps/s", "steps": K, "warmup": warmup,
           "ms_per_step": elapsed / K * 1e3, "players": n, "boards_per_gpu": B, "moves_per_launch": chunk,
           "roofline": {"bound": "valu-latency", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "kernel": f"k_rollout<{n}>", "kernel_avg_us": kernel_ms * 1e3,
                        "algorithmic_bytes_per_board_step": step_b,
                        "algorithmic_bytes_per_launch": step_b * B * chunk,
                        "moved_bytes_per_launch": moved * B, "moved_gbs": moved_gbs,
                        "moved_frac": moved_gbs / HBM_PEAK_GBS,
                        "limiter": "VALU issue + per-move dependency chains (PMC: ~22-25 % of VALU issue peak, "
                                   "~10 % of HBM); boards stay on chip for the launch, so 'achieved' is the "
                                   "SURVEY 8(d) algorithmic rate of a one-kernel-per-step design",
                        "pmc": issue},
           "games_completed": games, "untimed_ramp_launches": ramp}
    if cpu:
        rec["cpu_baseline"] = cpu_baseline(n, args.seed)
    return rec


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc, argv):
    """`bench.py --gpus N` outside torch.distributed.run (no WORLD_SIZE in the environment):
    start N ranks as one child torch.distributed.run on this node (127.0.0.1 rendezvous) and
    return its exit code. Runs before anything touches the GPU: the parent only waits; rank
    0 of the child prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    log(f"launching {nproc} ranks: {' '.join(cmd[1:6])} ...")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def dry_run(args, rank, world):
    """--dry-run: the multi-rank plumbing of the bench line without a GPU (gloo): barrier, a
    timed no-op interval, max over ranks, the episode-end example all-gather (splendor.
    selfplay.gather_examples over a few synthetic examples per rank, as config 4's window
    gathers), rank 0 prints the line (values null) with the record of each workload the run
    would measure at this N."""
    import torch.distributed as dist
    from splendor.selfplay import gather_examples
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    k = 3 + rank                                         # synthetic examples of this rank
    R = 32 + 10 * 2 + 4
    ex = {"board": torch.zeros((k, R, 7), dtype=torch.int8), "pi": torch.zeros((k, 409)),
          "meta": torch.full((k, 4), rank, dtype=torch.int32)}
    gathered = int(gather_examples(ex)["board"].shape[0])

    def record(cfg):
        n, B, sims = CONFIGS[cfg]
        return {"workload": cfg, "value": None, "n_gpus": world, "global_games": world * B, "numMCTSSims": sims,
                "window": {"examples_drained": k, "examples_gathered": gathered, **PHASES[cfg]}}
    head = "config3" if args.workload in ("all", "selfplay") else args.workload
    extra = {}
    if args.workload == "all" and world > 1 and not args.no_secondary:
        extra["config4_shard"] = record("config4")
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "rollouts/s (MCTS simulations)",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dry_run": True,
                          "ranks_reporting": world, "max_elapsed_s": elapsed,
                          "config": {"workload": head, "global_games": world * CONFIGS[head][1],
                                     "parallelism": f"dp{world} (game shards; RCCL all-gather of examples)"},
                          "selfplay": record(head), **extra}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000, help="timed self-play iterations (headline)")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--prefill", type=int, default=None, help="untimed iterations to the steady state first "
                    "(default: the workload's, PHASES)")
    ap.add_argument("--stagger", type=int, default=None, help="prefill iterations over which the games' phases "
                    "are spread (run_selfplay; ~ the mean game length: config 3 ~4,800 iterations)")
    ap.add_argument("--window", type=int, default=None, help="statistics window after the timed steps")
    ap.add_argument("--boards", type=int, default=32768, help="env workload: boards per GPU")
    ap.add_argument("--players", type=int, default=2, help="env workload: players")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--workload", choices=("all", "selfplay", "env", "config3", "config4", "config5"), default="all",
                    help="all: config-3 headline + config 2/5/4 objects (N=1); selfplay = config3 alone")
    ap.add_argument("--no-secondary", action="store_true", help="all: the headline only")
    ap.add_argument("--chunk", type=int, default=100, help="env: moves per rollout launch")
    ap.add_argument("--env-steps", type=int, default=1000, help="config-2 object: timed moves")
    ap.add_argument("--c5-prefill", type=int, default=PHASES["config5"]["prefill"])
    ap.add_argument("--c5-stagger", type=int, default=PHASES["config5"]["stagger"])
    ap.add_argument("--c5-window", type=int, default=PHASES["config5"]["window"])
    ap.add_argument("--c4-prefill", type=int, default=PHASES["config4"]["prefill"])
    ap.add_argument("--c4-stagger", type=int, default=PHASES["config4"]["stagger"])
    ap.add_argument("--c4-window", type=int, default=PHASES["config4"]["window"])
    ap.add_argument("--node-boards", type=int, default=-1, help="selfplay: 1/0 force node boards on/off "
                    "(default: on unless the pools do not fit)")
    ap.add_argument("--mem-gib", type=float, default=0.0, help="selfplay: arena budget in GiB (default: "
                    "BatchedMCTS.MEM_FRACTION of the free HBM)")
    ap.add_argument("--net", default=None, help="selfplay headline: a trained network (state_dict checkpoint, "
                    "tools/train_prior.py) instead of the random-init one")
    ap.add_argument("--dry-run", action="store_true", help="multi-rank plumbing only (gloo, no GPU): "
                    "prints the line with value null")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))    # the parent never touches the GPU
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        dry_run(args, rank, world)
        return
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    t_start = time.perf_counter()

    if args.workload == "env":
        rec = run_env(args, rank, world, dev, dist, args.steps, args.warmup,
                      cpu=rank == 0 and world == 1 and not args.no_cpu_baseline)
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": rec["value"], "unit": rec["unit"], "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": rec["ms_per_step"],
                              "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
                              "data": "synthetic (Philox-seeded deals, uniform-random legal actions)",
                              "config": {"workload": rec["workload"], "players": rec["players"],
                                         "boards_per_gpu": rec["boards_per_gpu"],
                                         "parallelism": f"dp{world} (board shards, no data-path collective)"},
                              "roofline": rec["roofline"], "cpu_baseline": rec.get("cpu_baseline")}))
        if dist:
            dist.destroy_process_group()
        return

    head = "config3" if args.workload in ("all", "selfplay") else args.workload
    n, B, sims = CONFIGS[head]
    ph = {k: (getattr(args, k) if getattr(args, k) is not None else v) for k, v in PHASES[head].items()}
    r = run_selfplay(head, rank, world, dev, dist, args.steps, args.warmup, ph["prefill"], ph["window"], args.seed,
                     args.node_boards, stagger=ph["stagger"], mem_gib=args.mem_gib, net_path=args.net)
    rec = selfplay_record(head, r, world, args.steps, args.warmup)
    torch.cuda.empty_cache()
    extra = {}
    secondary = args.workload == "all" and not args.no_secondary
    cpu_ok = rank == 0 and world == 1 and not args.no_cpu_baseline
    if cpu_ok:
        rec["cpu_baseline"] = cpu_baseline_selfplay(n, args.seed, sims)
    if secondary and world > 1:
        # BASELINE config 4 proper: 32,768 games per GPU (262,144 on 8), 1,600 simulations,
        # the examples all-gathered over RCCL at the end of its window (Coach.py:117-124)
        rr = run_selfplay("config4", rank, world, dev, dist, 1000, 100, args.c4_prefill, args.c4_window, args.seed,
                          args.node_boards, stagger=args.c4_stagger)
        extra["config4_shard"] = selfplay_record("config4", rr, world, 1000, 100)
        torch.cuda.empty_cache()
    elif secondary:
        extra["config2_env"] = run_env(args, rank, world, dev, dist, args.env_steps, 100, cpu=cpu_ok)
        for cfg, pf, sg, win in (("config5", args.c5_prefill, args.c5_stagger, args.c5_window),
                                 ("config4", args.c4_prefill, args.c4_stagger, args.c4_window)):
            rr = run_selfplay(cfg, rank, world, dev, dist, 1000, 100, pf, win, args.seed, args.node_boards, stagger=sg)
            o = selfplay_record(cfg, rr, world, 1000, 100)
            if cpu_ok:
                o["cpu_baseline"] = cpu_baseline_selfplay(CONFIGS[cfg][0], args.seed, CONFIGS[cfg][2],
                                                          target_s=2.0 if cfg == "config4" else 4.0)
            extra[{"config5": "config5_selfplay", "config4": "config4_shard"}[cfg]] = o
            torch.cuda.empty_cache()
    if rank == 0:
        cpu = rec.get("cpu_baseline")
        out = {
            "metric": METRIC, "value": rec["value"], "unit": "rollouts/s (MCTS simulations)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": rec["ms_per_iteration"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32 (network) / int8 (boards) / f64 (tree statistics)",
            "data": ("synthetic (Philox-seeded deals), random-init SplendorNNet (genbu.pt is refused by the "
                     "weights-only loader)") if not args.net else
                    f"synthetic (Philox-seeded deals), SplendorNNet trained by tools/train_prior.py ({args.net})",
            "config": {"workload": rec["workload"], "players": n, "games_per_gpu": B, "global_games": world * B,
                       "numMCTSSims": sims, "prefill_iterations": ph["prefill"],
                       "phase_stagger_iterations": ph["stagger"],
                       "parallelism": f"dp{world} (game shards; RCCL all-gather of examples)"},
            "roofline": selfplay_roofline(rec, n, rec["tree"]["leaf_depth_mean"]),
            "cpu_baseline": cpu,
            "selfplay": rec,
            **extra,
            "bench_seconds": time.perf_counter() - t_start,
        }
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
