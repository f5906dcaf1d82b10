"""GPU parity of the batched self-play driver (Coach.executeEpisode on device) against the
oracle's sequential self-play loop (same Philox decisions and Dirichlet draws, hash
network) and against whole reference episodes recorded with the same draws injected
(tests/golden/episode_*.npz). Bit-exact boards, per-game counters and every finished
training example."""
import os

import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import _oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


def make(n, B, sims, ratio, prob_full, forced, tthr=10, seed=9, **kw):
    from splendor.env import SplendorEngine
    from splendor.selfplay import SelfPlay
    args = dict(numMCTSSims=sims, cpuct=1.5, fpu=0.1, prob_fullMCTS=prob_full, ratio_fullMCTS=ratio,
                forced_playouts=forced, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=tthr)
    e = SplendorEngine(n)
    sp = SelfPlay(e, B, args, dirichlet_noise=kw.pop("noise", False), seed=seed, **kw)
    sp.reset()
    return e, sp


def sort_examples(ex, meta):
    order = np.lexsort((meta[:, 2], meta[:, 1], meta[:, 0]))
    return {k: v[order] for k, v in ex.items() if hasattr(v, "shape") and v.shape[:1] == meta.shape[:1]}


@pytest.mark.parametrize("n,forced,graph,noise,boards", [(2, False, False, False, True), (2, True, True, False, True),
                                                         (4, False, False, False, True), (2, False, True, True, True),
                                                         (4, True, True, True, True), (3, False, True, True, True),
                                                         (2, True, True, True, False), (3, False, True, True, False)])
def test_selfplay_matches_oracle(n, forced, graph, noise, boards):
    """boards: node boards kept (the descent follows linked edges without transitions) or
    not (the transition at every level) — identical results either way."""
    B, iters, sims, ratio, pf, seed = 96, 1200, 8, 4, 0.25, 9
    e, sp = make(n, B, sims, ratio, pf, forced, seed=seed, out_cap=20000, noise=noise, node_boards=boards)
    if graph:
        sp.run(iters - 3, use_graph=True)     # 8-iteration graph replays + single replays
        for _ in range(3):
            sp.step(use_graph=True)
    else:
        for _ in range(iters):
            sp.step(use_graph=False)
    torch.cuda.synchronize()
    hdr = sp.headers()
    assert hdr["overflow"].max() == 0
    ref = O.selfplay_run(n, B, iters, seed, sims, ratio, pf, 1.5, 0.1, forced, 10,
                         dir_alpha=0.3 if noise else 0.0, dir_temp=1.25)
    rh = ref["hdr"]
    np.testing.assert_array_equal(hdr["player"], rh[:, 0])
    np.testing.assert_array_equal(hdr["episode_step"], rh[:, 1])
    np.testing.assert_array_equal(hdr["move_no"], rh[:, 2])
    np.testing.assert_array_equal(hdr["game_no"], rh[:, 3])
    np.testing.assert_array_equal(hdr["games_done"], rh[:, 4])
    np.testing.assert_array_equal(hdr["sims_done"], rh[:, 6])
    np.testing.assert_array_equal(hdr["moves"], rh[:, 5])
    ex = {k: v.cpu().numpy() for k, v in sp.drain().items()}
    assert len(ex["pi"]) == len(ref["pi"]) > 0
    # the device queue order is nondeterministic: order both sides by (board id, game, index)
    ex = sort_examples(ex, ex["meta"])
    rf = sort_examples(ref, ref["meta"])
    np.testing.assert_array_equal(ex["meta"], rf["meta"])
    np.testing.assert_array_equal(ex["board"], rf["ex_board"])
    np.testing.assert_array_equal(ex["pi"], rf["pi"])
    np.testing.assert_array_equal(ex["valids"].view(np.uint64), rf["valids"])
    np.testing.assert_array_equal(ex["winner"], rf["winner"])
    np.testing.assert_array_equal(ex["scdiff"], rf["scdiff"])
    np.testing.assert_array_equal(ex["surprise"], rf["surprise"])


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("tag", ("2p", "2p_forced", "4p"))
def test_episode_matches_reference(tag):
    """Whole reference episodes (Coach.executeEpisode with root noise, temperature sampling,
    chance, symmetries; recorded with the build's keyed draws injected) replayed by the
    device self-play driver on one tree per recorded board id, examples expanded by the
    device symmetry kernel: the reference's example list, bit for bit."""
    from splendor.coach import expand_symmetries
    from splendor.env import unpack_mask
    with np.load(os.path.join(GOLD, f"episode_{tag}.npz")) as z:
        d = {k: z[k] for k in z.files}
    n = {56: 2, 71: 3, 88: 4}[d["board"].shape[1]]
    a = {k[4:]: d[k] for k in d if k.startswith("arg_")}
    sims, ratio = int(a["numMCTSSims"]), int(a["ratio_fullMCTS"])
    for gi, gb in enumerate(d["game_board_id"]):
        e, sp = make(n, 1, sims, ratio, float(a["prob_fullMCTS"]), bool(a["forced_playouts"]),
                     tthr=int(a["tempThreshold"]), seed=int(d["seed"]), board_base=int(gb), noise=True,
                     out_cap=4096)
        assert float(a["cpuct"]) == 1.5 and float(a["fpu"]) == 0.1 and float(a["dirichletAlpha"]) == 0.3
        moves = 0
        while sp.stats()["games_done"] == 0:
            sp.run(256, use_graph=True)
            moves += 1
            assert moves < 64, "episode did not finish"
        ex = sp.drain()
        keep = ex["meta"][:, 1] == 0
        ex = {k: v[keep] for k, v in ex.items()}
        order = torch.argsort(ex["meta"][:, 2])
        ex = expand_symmetries(e, {k: v[order] for k, v in ex.items()})
        sel = d["game"] == gi
        assert ex["board"].shape[0] == int(sel.sum()) == int(d["game_n_examples"][gi])
        np.testing.assert_array_equal(ex["board"].cpu().numpy(), d["board"][sel])
        np.testing.assert_array_equal(ex["pi"].cpu().numpy(), d["pi"][sel])
        np.testing.assert_array_equal(unpack_mask(ex["valids"]).cpu().numpy().astype(np.uint8), d["valids"][sel])
        np.testing.assert_array_equal(ex["winner"].cpu().numpy(), d["winner"][sel])
        np.testing.assert_array_equal(ex["scdiff"].cpu().numpy(), d["scdiff"][sel])
        np.testing.assert_array_equal(ex["surprise"].cpu().numpy(), d["surprise"][sel].astype(np.float32))


def test_selfplay_with_noise_and_network_sane():
    from splendor.env import unpack_mask
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.env import SplendorEngine
    from splendor.selfplay import SelfPlay
    e = SplendorEngine(2)
    B = 512
    args = dict(numMCTSSims=25, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5,
                forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    ev = LeafEvaluator(e, random_net(2, seed=0), B)
    sp = SelfPlay(e, B, args, evaluator=ev, dirichlet_noise=True, seed=3)
    sp.reset()
    for _ in range(400):
        sp.step(use_graph=True)
    st = sp.stats()
    assert st["overflow"] == 0 and st["moves"] > B
    ex = sp.drain()
    if len(ex["pi"]):
        pi = ex["pi"].double()
        assert torch.allclose(pi.sum(1), torch.ones_like(pi.sum(1)), atol=1e-5)
        valid = unpack_mask(ex["valids"])
        assert bool((pi[~valid] == 0).all())
        assert set(np.unique(ex["winner"].cpu().numpy()).tolist()) <= {-1.0, 1.0, np.float32(0.01)}


def test_iteration_examples_roundtrip(tmp_path):
    """Coach.executeIteration -> ExampleSet (columnar, symmetries expanded on device) ->
    checkpoint.examples.npz -> identical tuples to the reference-format executeEpisodes."""
    from splendor.SplendorGame import SplendorGame
    from splendor.coach import Coach
    from splendor.mcts import HashEvaluator
    args = dict(numMCTSSims=8, cpuct=1.5, fpu=0.1, prob_fullMCTS=1.0, ratio_fullMCTS=4,
                forced_playouts=False, dirichletAlpha=0.0, temperature=[1.25, 0.8], tempThreshold=10,
                numItersHistory=3, checkpoint=str(tmp_path))

    def coach():
        g = SplendorGame(2)
        c = Coach(g, None, args, batch=32, seed=5)
        c.sp.evaluator = HashEvaluator(g.engine)
        return c

    a = coach()
    exset = a.executeIteration(4)
    assert len(exset) > 0 and len(a.trainExamplesHistory.iters) == 1
    ref = coach().executeEpisodes(4)                    # reference tuple form, same seeds
    key = lambda t: (t[0].tobytes(), t[1].tobytes())
    got = sorted(exset.to_tuples(), key=key)
    ref = sorted(ref, key=key)
    assert len(got) == len(ref)
    for x, y in zip(got, ref):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(u, v)
    path = a.saveTrainExamples()
    b = coach()
    b.loadTrainExamples(str(tmp_path))
    back = b.trainExamplesHistory.merged()
    for k in ("board", "pi", "winner", "scdiff", "valids", "surprise"):
        assert torch.equal(getattr(back, k).cpu(), getattr(exset, k).cpu()), k
    assert path.endswith("checkpoint.examples.npz")


def test_train_on_device_examples():
    """Self-play examples stay on the device into NNetWrapper.train (GenericNNetWrapper
    .train with columnar inputs), and the trained weights drive the next search."""
    from splendor.NNet import NNetWrapper
    from splendor.SplendorGame import SplendorGame
    from splendor.coach import Coach
    g = SplendorGame(2)
    nn = NNetWrapper(g, dict(epochs=1, batch_size=32))
    args = dict(numMCTSSims=8, cpuct=2.5, fpu=0.3, prob_fullMCTS=1.0, ratio_fullMCTS=4,
                forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    c = Coach(g, nn, args, batch=64, seed=2)
    exset = c.executeIteration(8)
    assert exset.board.is_cuda and len(exset) >= 32
    before = [p.detach().clone() for p in nn.nnet.parameters()]
    out = nn.train(exset)
    assert all(np.isfinite(v) for v in out.values())
    assert any(not torch.equal(a, b) for a, b in zip(before, nn.nnet.parameters()))
    c2 = Coach(g, nn, args, batch=16, seed=3)          # evaluator packs the trained weights
    c2.run_iterations(4)
    assert c2.sp.stats()["overflow"] == 0


def test_full_size_selfplay_invariants():
    """BASELINE config 3 size (32,768 games, genbu args, SplendorNNet leaves): after every
    iteration batch, each tree's root visit counts cover its finished simulations, every
    visited Q lies in [-1, 1] (unvisited = the reference's -42), and moves get committed."""
    from splendor.env import SplendorEngine
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.selfplay import SelfPlay
    B = 32768
    args = dict(numMCTSSims=100, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5,
                forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    e = SplendorEngine(2)
    sp = SelfPlay(e, B, args, evaluator=LeafEvaluator(e, random_net(2, seed=0), B, use_graph=False),
                  dirichlet_noise=True, seed=17)
    sp.reset()
    for rep in range(3):
        for _ in range(40):
            sp.step(use_graph=True)
        torch.cuda.synchronize()
        h = sp.headers()
        assert (h["overflow"] == 0).all()
        counts, qsa, _, _ = sp.root_stats()
        sims = torch.from_numpy(h["sims_done"].astype(np.int64)).cuda()
        has_root = torch.from_numpy(h["root"] >= 0).cuda()
        # every simulation of the current search passes one root edge (except the root's own
        # expansion when the root is new); a kept root also carries its earlier visits
        tot = counts.sum(1)
        assert bool((tot[has_root] >= sims[has_root] - 1).all()), rep
        visited = counts > 0
        assert bool(((qsa[visited] >= -1.0) & (qsa[visited] <= 1.0)).all())
        assert bool((qsa[~visited] == -42.0).all())
    st = sp.stats()
    assert st["moves"] > B                              # moves were committed on every tree


def test_coach_learn_iteration(tmp_path):
    """Coach.learn (Coach.py:102-164) end to end on the engine, tiny: self-play games,
    example history file, one training pass, the BatchedArena gate and checkpoints."""
    import os
    from splendor.NNet import NNetWrapper
    from splendor.SplendorGame import SplendorGame
    from splendor.coach import Coach
    g = SplendorGame(2)
    nn = NNetWrapper(g, dict(epochs=1, batch_size=32))
    args = dict(numMCTSSims=6, cpuct=2.5, fpu=0.3, prob_fullMCTS=1.0, ratio_fullMCTS=3,
                forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10,
                numIters=1, numEps=4, numItersHistory=2, arenaCompare=4, updateThreshold=0.55,
                checkpoint=str(tmp_path))
    c = Coach(g, nn, args, batch=32, seed=4)
    hist = c.learn()
    assert len(hist) == 1
    nwins, pwins, draws, ok = hist[0]
    assert nwins + pwins + draws == 4
    files = set(os.listdir(tmp_path))
    assert {"temp.pt", "checkpoint.examples.npz"} <= files
    assert ("best.pt" in files) == ok
    assert len(c.trainExamplesHistory.iters) == 1 and len(c.trainExamplesHistory) > 0


@pytest.mark.gpu
def test_compacted_leaf_evaluation_matches_full_batch():
    """Self-play with the network evaluated on the compacted NN-leaf list
    (spl_mcts_select_compact + spl_nn_forward_indexed) plays exactly the games of the
    full-batch evaluation: headers, root counts and drained examples bit-identical."""
    from splendor.env import SplendorEngine
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.selfplay import SelfPlay
    args = dict(numMCTSSims=24, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.5, ratio_fullMCTS=4, forced_playouts=False,
                dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
    e = SplendorEngine(2)
    net = random_net(2, seed=1)
    out = []
    for indexed in (True, False):
        ev = LeafEvaluator(e, net, 256, use_graph=False)
        if not indexed:
            ev.__class__ = type("FullBatch", (LeafEvaluator,), {"indexed": property(lambda self: False)})
        sp = SelfPlay(e, 256, args, evaluator=ev, seed=0x5EED)
        sp.reset()
        sp.run(1500, use_graph=True)
        torch.cuda.synchronize()
        h = sp.headers()
        ex = sp.drain()
        out.append((h, sp.root_stats()[0].cpu().numpy(), {k: v.cpu().numpy() for k, v in ex.items()}))
        del sp
    (h0, c0, e0), (h1, c1, e1) = out
    for k in ("player", "episode_step", "move_no", "game_no", "games_done", "moves", "sims_done", "depth"):
        np.testing.assert_array_equal(h0[k], h1[k], err_msg=k)
    np.testing.assert_array_equal(c0, c1)
    assert len(e0["meta"]) > 0
    o0, o1 = np.lexsort(e0["meta"].T[::-1]), np.lexsort(e1["meta"].T[::-1])
    for k in e0:
        np.testing.assert_array_equal(e0[k][o0], e1[k][o1], err_msg=k)


def test_restart_games_abandons_only_the_chosen_games():
    """spl_mcts_restart_games (bench.py's phase stagger): the chosen trees abandon their game
    (staged examples discarded, nothing queued) and start their next one (game number + 1,
    a fresh tree and search); every other tree is untouched and plays on."""
    B = 96
    e, sp = make(2, B, 8, 4, 0.25, False, out_cap=40000)
    sp.run(150, use_graph=False)
    torch.cuda.synchronize()
    before = sp.headers().copy()
    queued = sp.drain()
    chosen = np.arange(B) % 3 == 1
    sp.restart(torch.from_numpy(chosen))
    torch.cuda.synchronize()
    after = sp.headers()
    assert sp.drain()["board"].shape[0] == 0                 # nothing queued by a restart
    for k in ("game_no",):
        np.testing.assert_array_equal(after[k][chosen], before[k][chosen] + 1)
    for k in ("episode_step", "player", "n_examples", "sims_done", "node_count"):
        assert (after[k][chosen] == 0).all(), k
    assert (after["budget"][chosen] > 0).all()
    keep = ~chosen
    for k in HDR_KEYS:
        np.testing.assert_array_equal(after[k][keep], before[k][keep], err_msg=k)
    sp.run(400, use_graph=False)
    torch.cuda.synchronize()
    h = sp.headers()
    assert h["overflow"].max() == 0 and h["unexpanded"].max() == 0
    ex = sp.drain()
    meta = ex["meta"].cpu().numpy()
    # examples of the restarted boards only come from games dealt after the restart
    for t in np.nonzero(chosen)[0]:
        g = meta[meta[:, 0] == t, 1]
        assert (g > before["game_no"][t] - 1).all() or g.size == 0
    assert queued["board"].shape[0] + ex["board"].shape[0] > 0


HDR_KEYS = ("node_count", "edge_count", "root", "sims_done", "budget", "full", "player", "episode_step",
            "move_no", "game_no", "n_examples", "games_done", "moves")


GENBU = dict(cpuct=2.5, fpu=0.3, prob_full=0.25, ratio=5, noise=True)


def _deep_device(n, B, iters, sims=100, seed=11, mode=1, **kw):
    from splendor.env import SplendorEngine
    from splendor.mcts import HashEvaluator
    from splendor.selfplay import SelfPlay
    args = dict(numMCTSSims=sims, cpuct=GENBU["cpuct"], fpu=GENBU["fpu"], prob_fullMCTS=GENBU["prob_full"],
                ratio_fullMCTS=GENBU["ratio"], forced_playouts=False, dirichletAlpha=0.3, temperature=[1.25, 0.8],
                tempThreshold=10)
    e = SplendorEngine(n)
    sp = SelfPlay(e, B, args, evaluator=HashEvaluator(e, mode=mode), dirichlet_noise=True, seed=seed,
                  out_cap=60000, **kw)
    sp.reset()
    sp.run(iters, use_graph=True)
    torch.cuda.synchronize()
    hdr = sp.headers()
    st = sp.stats()
    ex = {k: v.cpu().numpy() for k, v in sp.drain().items()}
    print(f"deep self-play n={n} B={B} iters={iters} {kw}: {st}", flush=True)
    del sp
    return hdr, st, ex


def _oracle_lagged(n, B, iters, seed, sims, lag, mode=1):
    """The oracle's self-play loop (peaked hash network, genbu arguments) where tree t runs
    iters - lag[t] iterations: a withdrawn simulation repeats in the next iteration, so a tree
    that withdrew w times is exactly w simulations behind. Board-id parts run in worker
    processes (every draw is keyed by the global board id)."""
    args = (sims, GENBU["ratio"], GENBU["prob_full"], GENBU["cpuct"], GENBU["fpu"], False, 10)
    return O.selfplay_run_parallel(n, B, iters, seed, *args, lag=lag, max_ex=60000, dir_alpha=0.3, dir_temp=1.25,
                                   fake_mode=mode)


def _deep_selfplay(n, B, iters, sims=100, seed=11, device_run=None, mode=1, **kw):
    """Self-play with the peaked hash network (mode 1: the random-init SplendorNNet's regime:
    deep trees, long terminal lines) against the oracle's sequential loop, bit for bit."""
    hdr, st, ex = device_run or _deep_device(n, B, iters, sims, seed, mode=mode, **kw)
    t0 = time.perf_counter()
    ref = _oracle_lagged(n, B, iters, seed, sims, hdr["withdrawals"], mode=mode)
    print(f"oracle: {time.perf_counter() - t0:.1f} s", flush=True)
    rh = ref["hdr"]
    for k, j in (("player", 0), ("episode_step", 1), ("move_no", 2), ("game_no", 3), ("games_done", 4),
                 ("moves", 5), ("sims_done", 6)):
        np.testing.assert_array_equal(hdr[k], rh[:, j], err_msg=k)
    dsum, dmax, dcnt = ref["depth"]
    assert st["depth_sum"] == dsum and st["depth_max_all"] == dmax     # every simulation's leaf depth
    assert len(ex["pi"]) == len(ref["pi"])
    if not len(ex["pi"]):
        return st, dsum / dcnt, dmax
    ex = sort_examples(ex, ex["meta"])
    rf = sort_examples(ref, ref["meta"])
    for k, rk in (("meta", "meta"), ("board", "ex_board"), ("pi", "pi"), ("winner", "winner"),
                  ("scdiff", "scdiff"), ("surprise", "surprise")):
        np.testing.assert_array_equal(ex[k], rf[rk], err_msg=k)
    np.testing.assert_array_equal(ex["valids"].view(np.uint64), rf["valids"])
    return st, dsum / dcnt, dmax


@pytest.mark.parametrize("n,B,iters", [(2, 128, 3000), (4, 64, 2000)])    # (4p games outlast 2,000)
def test_deep_selfplay_matches_oracle(n, B, iters):
    """The bench's regime: genbu search arguments, Dirichlet noise, 100
    simulations, the peaked hash network — leaves at mean depth > 15 and beyond 64 levels, so
    k_backup's later 64-level groups and the descent's path reuse past 64 levels run — bit
    for bit against the oracle (headers, every leaf depth, every finished example)."""
    st, mean, mx = _deep_selfplay(n, B, iters)
    assert mean > 15 and mx > 64, (mean, mx)
    assert st["prunes"] == st["resets"] == st["unexpanded"] == 0


@pytest.mark.parametrize("n,sims,iters,mode", [(2, 1600, 90000, 1), (2, 1600, 90000, 0), (4, 400, 45000, 1),
                                               (4, 400, 45000, 0)])
def test_large_budget_selfplay_matches_oracle(n, sims, iters, mode):
    """BASELINE configs 4 (2p, numMCTSSims 1,600) and 5 (4p, 400) at their search budgets
    (MCTS.py:45-60 full / fast searches, :99-177, :199-219): 32 games of self-play with genbu's
    arguments and Dirichlet noise, long enough for the games to finish (2p: up to 124 moves of
    ~640 simulations; 4p: 248 of ~160), bit for bit against the oracle — headers, every
    simulation's leaf depth, every finished example (board, pi, winner, scdiff, surprise,
    valids). Two hash networks: the peaked one (mode 1: deep trees, leaves past 64 levels) and
    the spread one (mode 0: wide nodes — the peaked network never gives a non-root node more
    than 12 visited edges). Asserted to have run, from the device's counters: visit blocks
    relocated to 128 or more records (both), and (mode 0) non-root levels with more than 12
    visit records evaluated exactly."""
    B = 32
    t0 = time.perf_counter()
    run = _deep_device(n, B, iters, sims=sims, mode=mode, mem_budget=16 << 30)
    print(f"device: {time.perf_counter() - t0:.1f} s", flush=True)
    st, mean, mx = _deep_selfplay(n, B, iters, sims=sims, device_run=run, mode=mode)
    print(f"large budget n={n} sims={sims} mode={mode}: mean leaf depth {mean:.1f}, max {mx}, {st}", flush=True)
    assert st["games_done"] >= B // 2
    assert st["prunes"] == st["resets"] == st["unexpanded"] == 0
    assert st["big_moves"] > 0, "no visit block was relocated to 128 or more records"
    if mode == 1:
        assert mean > 15 and mx > 64, (mean, mx)
    else:
        assert st["exact_wide"] > 0, "no non-root level with more than 12 visit records was evaluated exactly"


def test_withdrawals_repeat_the_same_simulation():
    """Shared pools sized so searches run out of pages mid-search: the leaf is withdrawn,
    k_gc collects the tree's garbage and the descent repeats — the games stay bit-exact with
    the oracle's (which never runs out), with withdrawals > 0 and no other capacity event.
    The pools shrink step by step (device only) until a run withdraws without any other
    event; that run is compared with the oracle."""
    from splendor.mcts import BatchedMCTS
    n, B, iters = 2, 64, 2000
    nc = BatchedMCTS.default_node_cap(100)
    ratio = BatchedMCTS.UNITS_PER_NODE

    def run(per_tree):
        return _deep_device(n, B, iters, pool_nodes=B * per_tree, pool_edges=B * per_tree * ratio,
                            node_cap=nc, edge_cap=32 * nc)

    def events(r):
        return r[1]["withdrawals"], r[1]["prunes"] + r[1]["resets"] + r[1]["unexpanded"]
    hi, lo, found = 4096, None, None        # hi: no withdrawals; lo: withdrawals with other events
    for per_tree in (2048, 1024, 512, 256):
        r = run(per_tree)
        w, other = events(r)
        if w and not other:
            found = r
            break
        if w:
            lo = per_tree
            break
        hi = per_tree
    while found is None and lo is not None and hi - lo > 4:
        mid = (hi + lo) // 2
        r = run(mid)
        w, other = events(r)
        if w and not other:
            found = r
        elif w:
            lo = mid
        else:
            hi = mid
    assert found is not None, "no pool size gave withdrawals without other capacity events"
    st, _, _ = _deep_selfplay(n, B, iters, device_run=found)
    assert st["withdrawals"] > 0
