"""BASELINE configs 4 and 5 on the GPU, and device sharding.

* Sharding: every random draw is keyed by the global board id, so a shard of B' boards at
  board_base = k * B' must reproduce, bit for bit, the matching slice of one launch over
  all boards — for the fused rollout kernel (config 2) and for batched self-play (configs
  3-5). This is what makes results independent of the GPU count.
* Config 5 (4 players, 16,384 games, numMCTSSims=400, Dirichlet on): full-size self-play
  with SplendorNNet leaves (property checks), and the slice equality plus the oracle on a
  64-game slice with the hash network (bit-exact, noise included).
* Config 4 per-GPU shard (2 players, 32,768 games, numMCTSSims=1600): full size with pools
  planned against the device's memory, run past its steady state (phase-spread, as the
  bench) with zero capacity events; searches keep running under capacity pressure (events
  counted, never a frozen tree), and the slice equality with the hash network.
"""
import gc
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import _oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GENBU = dict(cpuct=2.5, fpu=0.3, prob_fullMCTS=0.25, ratio_fullMCTS=5, forced_playouts=False,
             dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)
HDR_KEYS = ("player", "episode_step", "move_no", "game_no", "games_done", "sims_done", "budget", "full",
            "moves", "prunes", "resets", "unexpanded")
# (slot counts and root ids are not compared: trees share the per-GPU pools, so which pages a
# tree holds and how much garbage it carries depend on the other trees; the live table —
# root + nodes beyond the root's round, and their edges — does not)


def free_all():
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_rollout_shard_equals_slice():
    """Config 2: 32,768 boards in one launch vs a 512-board shard at board_base 20,480."""
    from splendor.env import RolloutBatch, SplendorEngine
    e = SplendorEngine(2)
    B, b0, Bs, K = 32768, 20480, 512, 150
    full = RolloutBatch(e, B, seed=0x5EED)
    fo = full.run(K)
    shard = RolloutBatch(e, Bs, seed=0x5EED, board_base=b0)
    so = shard.run(K)
    torch.cuda.synchronize()
    sl = slice(b0, b0 + Bs)
    assert torch.equal(full.state[sl], shard.state)
    assert torch.equal(full.player[sl], shard.player)
    assert torch.equal(full.games[sl], shard.games)
    assert torch.equal(fo["action"][:, sl], so["action"])
    assert torch.equal(fo["mask"][:, sl], so["mask"])
    assert torch.equal(fo["ended"][:, sl], so["ended"])
    assert int(full.games.sum()) > 0


def selfplay(n, B, sims, board_base=0, evaluator=None, **kw):
    from splendor.env import SplendorEngine
    from splendor.mcts import HashEvaluator
    from splendor.selfplay import SelfPlay
    e = SplendorEngine(n)
    sp = SelfPlay(e, B, dict(GENBU, numMCTSSims=sims), evaluator=evaluator or HashEvaluator(e),
                  dirichlet_noise=True, seed=0x5EED, board_base=board_base, **kw)
    sp.reset()
    return e, sp


def assert_slice_equal(full, shard, b0):
    hf, hs = full.headers(), shard.headers()
    Bs = shard.B
    for k in HDR_KEYS:
        np.testing.assert_array_equal(hf[k][b0:b0 + Bs], hs[k], err_msg=k)
    np.testing.assert_array_equal(full.tree_sizes()[b0:b0 + Bs, 2:], shard.tree_sizes()[:, 2:], err_msg="live")
    np.testing.assert_array_equal(hf["root"][b0:b0 + Bs] >= 0, hs["root"] >= 0, err_msg="has root")
    assert torch.equal(full.root_stats()[0][b0:b0 + Bs], shard.root_stats()[0])
    assert torch.equal(full.root_priors()[b0:b0 + Bs], shard.root_priors())


def test_config5_shard_equals_slice_and_oracle():
    """4p, 16,384 games, 400 simulations, root noise: a 64-game shard equals the slice of
    the full batch, and the oracle's self-play on those 64 board ids (bit-exact)."""
    n, B, sims, iters, b0, Bs = 4, 16384, 400, 900, 8192, 64
    caps = dict(node_cap=4096, edge_cap=4096 * 48)
    _, full = selfplay(n, B, sims, **caps)
    full.run(iters, use_graph=True)
    _, shard = selfplay(n, Bs, sims, board_base=b0, **caps)
    shard.run(iters, use_graph=True)
    torch.cuda.synchronize()
    assert_slice_equal(full, shard, b0)
    st = full.stats()
    assert st["overflow"] == 0 and st["moves"] > B and st["unexpanded"] == 0
    assert st["prunes"] == st["resets"] == 0
    del full
    free_all()
    ref = O.selfplay_run_parallel(n, Bs, iters, 0x5EED, sims, GENBU["ratio_fullMCTS"], GENBU["prob_fullMCTS"],
                                  GENBU["cpuct"], GENBU["fpu"], False, GENBU["tempThreshold"], board_base=b0,
                                  dir_alpha=0.3, dir_temp=1.25)
    h = shard.headers()
    for j, k in enumerate(("player", "episode_step", "move_no", "game_no", "games_done", "moves", "sims_done", "budget")):
        np.testing.assert_array_equal(h[k], ref["hdr"][:, j], err_msg=k)
    ss = shard.stats()                          # every simulation's leaf depth (sum, maximum)
    assert (ss["depth_sum"], ss["depth_max_all"]) == ref["depth"][:2]
    # (the full example / pi comparison at this budget: test_selfplay_gpu.py::
    # test_large_budget_selfplay_matches_oracle[4-400-45000])


@pytest.mark.parametrize("n,B,sims,iters", [(4, 16384, 400, 1000), (2, 32768, 1600, 2400)])
def test_full_size_selfplay_with_network(n, B, sims, iters):
    """Configs 5 and 4 (per-GPU shard) at full size with SplendorNNet leaves and the default
    memory-planned pools: moves commit on every tree, root statistics are consistent, noised
    root priors sum to 1, no tree freezes; capacity events are reported."""
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.env import SplendorEngine
    e = SplendorEngine(n)
    ev = LeafEvaluator(e, random_net(n, seed=0), B, use_graph=False)
    free = torch.cuda.mem_get_info()[0]
    _, sp = selfplay(n, B, sims, evaluator=ev)
    assert sp.device_bytes <= 0.8 * free                      # planned against free memory
    sp.run(iters, use_graph=True)
    torch.cuda.synchronize()
    st = sp.stats()
    h = sp.headers()
    assert st["overflow"] == 0 and st["moves"] >= B
    counts, qsa, _, _ = sp.root_stats()
    has_root = torch.from_numpy(h["root"] >= 0).cuda()
    sims_done = torch.from_numpy(h["sims_done"].astype(np.int64)).cuda()
    assert bool((counts.sum(1)[has_root] >= sims_done[has_root] - 1).all())
    visited = counts > 0
    assert bool(((qsa[visited] >= -1.0) & (qsa[visited] <= 1.0)).all())
    ps = sp.root_priors()
    tot = ps.double().sum(1)[has_root]
    assert bool((torch.abs(tot - 1.0) < 1e-4).all())
    print(f"config n={n} B={B} sims={sims}: {st}, node_cap {sp.cfg.node_cap}, edge_cap {sp.cfg.edge_cap}, "
          f"device bytes {sp.device_bytes / 2**30:.1f} GiB")
    del sp, ev
    free_all()


def test_config4_shard_equals_slice():
    """2p, 32,768 games x 1,600 simulations (hash network): a 128-game shard at board_base
    24,576 equals the slice of the full batch (headers, root counts, root priors)."""
    n, B, sims, iters, b0, Bs = 2, 32768, 1600, 2000, 24576, 128
    caps = dict(node_cap=2560, edge_cap=2560 * 32)
    _, full = selfplay(n, B, sims, **caps)
    full.run(iters, use_graph=True)
    _, shard = selfplay(n, Bs, sims, board_base=b0, **caps)
    shard.run(iters, use_graph=True)
    torch.cuda.synchronize()
    assert_slice_equal(full, shard, b0)
    assert full.stats()["moves"] > B
    del full, shard
    free_all()


def test_capacity_pressure_is_graceful():
    """Pools far too small for the trees the reference would keep: searches start on pruned
    or emptied trees and leaves that do not fit are backed up without being stored — every
    game keeps playing, examples keep flowing, the events are counted."""
    n, B, sims = 2, 256, 64
    _, sp = selfplay(n, B, sims, node_cap=96, edge_cap=96 * 24)
    for _ in range(10):
        sp.run(400, use_graph=True)
        sp.drain()
    st = sp.stats()
    print("capacity pressure:", st)
    assert st["overflow"] == 0 and st["games_done"] > 0
    assert st["prunes"] > 0 and st["withdrawals"] > 0 and st["collections"] > 0
    h = sp.headers()
    nmax, epages = 128, 2                                        # caps rounded up to whole pages
    assert (h["node_count"] <= nmax).all() and (h["epg"] <= epages).all()   # (2,048-unit pages)
    assert h["moves"].min() > 10                                 # every tree kept committing moves
    # the GC queue drains: what stays queued is only "should" collections deferred to later
    # launches (GC_SHOULD_CAP per launch)
    assert ((h["gc_queued"] == 0) | (h["gc_state"] == 5)).all()


def test_search_arena_spends_whole_budget_under_pressure():
    """A search-only arena (BatchedMCTS, no self-play commit) whose trees cannot hold a
    search: no simulation is withdrawn (there is no lazy garbage to collect), leaves that do
    not fit are backed up unstored, and every tree spends exactly its budget."""
    from splendor.env import SplendorEngine
    from splendor.mcts import BatchedMCTS
    e = SplendorEngine(2)
    B, sims = 64, 200
    m = BatchedMCTS(e, B, dict(numMCTSSims=sims, cpuct=1.5, fpu=0.1), node_cap=64, edge_cap=1024)
    roots = e.new_state(B)
    e.init(roots, seed=7)
    m.set_roots(roots, keep_tree=False)
    m.search()
    h = m.headers()
    assert (h["sims_done"] == h["budget"]).all() and (h["budget"] == sims).all()
    assert (h["withdrawals"] == 0).all()
    assert m.capacity_events(h)["unexpanded"] > 0
    counts = m.root_stats()[0]
    assert bool((counts.sum(1) == sims - 1).all())


@pytest.mark.parametrize("n,B,sims,prefill,window,stagger", [(2, 32768, 100, 3000, 3000, 0),
                                                             (4, 16384, 400, 30000, 8000, 0),
                                                             (2, 32768, 1600, "bench", 4000, "bench")])
def test_steady_state_search_is_reference_exact(n, B, sims, prefill, window, stagger):
    """Configs 3, 5 and 4's per-GPU shard at full size with SplendorNNet leaves on the default
    shared pools, run to their steady state (config 3: games finish from ~2,400 iterations
    on; config 5: the first games end near 16,000 and the trees that all started together
    peak around 20,000; config 4: games spread over the phases of a game as in bench.py,
    `stagger`) and then through a window: no search in the window ran on a pruned or emptied
    tree and every leaf was stored (prunes == resets == unexpanded == 0), so each tree is the
    reference's table. Events during the start-up transient are printed."""
    import importlib.util
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.env import SplendorEngine
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    if prefill == "bench":                      # config 4: bench.py's own phases (~ one game)
        prefill, stagger = bench.PHASES["config4"]["prefill"], bench.PHASES["config4"]["stagger"]
    e = SplendorEngine(n)
    ev = LeafEvaluator(e, random_net(n, seed=0), B, use_graph=False)
    _, sp = selfplay(n, B, sims, evaluator=ev)

    def run(k):
        done = 0
        while done < k:
            sp.run(min(4000, k - done), use_graph=True)
            done += min(4000, k - done)
            sp.drain()
    done = 0
    for target, j in bench.stagger_marks(stagger, 16, sims, GENBU["ratio_fullMCTS"]) + [(prefill, None)]:
        run(target - done)                      # (phase stagger as bench.run_selfplay)
        done = target
        if j is not None:
            sp.restart(torch.arange(B) % 16 == j)
    ev0 = sp.check_capacity(allow=True)
    g0 = sp.stats()["games_done"]
    run(window)
    torch.cuda.synchronize()
    st = sp.stats()
    ev1 = sp.check_capacity(allow=True)
    pool = sp.pool_state()
    del sp, ev                                  # (freed before asserting: a failed test's
    free_all()                                  #  traceback must not pin ~230 GB of pools)
    delta = {k: ev1[k] - ev0[k] for k in ev1}
    print(f"steady state n={n} B={B} sims={sims}: start-up events {ev0}, window events {delta}, "
          f"window games {st['games_done'] - g0}, {st}, pool {pool}")
    assert st["games_done"] - g0 > 0 and st["overflow"] == 0
    assert delta == {"prunes": 0, "resets": 0, "unexpanded": 0}


def test_check_capacity_raises_on_events():
    """Capacity events are an error unless the caller allows them."""
    from splendor import _lib
    n, B, sims = 2, 64, 64
    _, sp = selfplay(n, B, sims, node_cap=96, edge_cap=96 * 24)
    sp.run(1200, use_graph=True)
    sp.drain()
    with pytest.raises(_lib.EngineError):
        sp.check_capacity()
    ev = sp.check_capacity(allow=True)
    assert ev["prunes"] > 0
