"""Batched device-resident MCTS (host side of csrc/mcts.hip).

`BatchedMCTS` holds B persistent search trees in HBM (one per board/game) and exposes the
reference's search API in batched form:

    reference (MCTS.py)                              here
    MCTS(game, nnet, args, dirichlet_noise)          BatchedMCTS(engine, B, args, evaluator)
    getActionProb(canonicalBoard, temp=1, full)      get_action_prob(canonical_boards, full)
    reset_all_search_trees()                         reset()

`evaluator(leaf_state int8[B,R,7], leaf_mask int64[B,7], leaf_valid uint8[B]) -> (pi
float32[B,409], v float32[B,n])` is the batched `nnet.predict` (GenericNNetWrapper.py:141):
`HashEvaluator` (deterministic, parity tests) or `splendor.nnet.NetEvaluator`
(SplendorNNet under PyTorch-ROCm).
"""
import ctypes as C

import numpy as np
import torch

from . import _lib
from .env import ACTIONS, MASK_WORDS, _ptr

# TreeHdr (csrc/mcts_device.h), 144 bytes
HDR_DTYPE = np.dtype([
    ("node_count", "<i4"), ("edge_count", "<i4"), ("root", "<i4"), ("sims_done", "<i4"),
    ("budget", "<i4"), ("full", "<i4"), ("noise_pending", "<i4"), ("depth", "<i4"),
    ("leaf_kind", "<i4"), ("player", "<i4"), ("episode_step", "<i4"), ("move_no", "<i4"),
    ("game_no", "<i4"), ("overflow", "<i4"), ("n_examples", "<i4"), ("leaf_round", "<i4"),
    ("leaf_k0", "<u8"), ("leaf_k1", "<u8"), ("leaf_v", "<f4", (4,)),
    ("games_done", "<i4"), ("forced", "<i4"), ("pad0", "<i4"), ("root_eb", "<i4"),
    ("prunes", "<i4"), ("resets", "<i4"), ("unexpanded", "<i4"), ("root_ec", "<i4"),
    ("gc_state", "<i4"), ("pad1", "<i4"), ("pad2", "<i4"), ("pad3", "<i4")])
assert HDR_DTYPE.itemsize == 144

DEFAULT_ARGS = dict(numMCTSSims=100, cpuct=1.0, fpu=0.0, prob_fullMCTS=1.0, ratio_fullMCTS=5,
                    forced_playouts=False, dirichletAlpha=0.0, temperature=[1.25, 0.8],
                    tempThreshold=10)


def _arg(args, k):
    if args is None:
        return DEFAULT_ARGS[k]
    try:
        return args[k]
    except (KeyError, TypeError):
        return getattr(args, k, DEFAULT_ARGS[k])


class HashEvaluator:
    """Deterministic stand-in network (spl_hash_eval); identical to the oracle's."""

    def __init__(self, engine):
        self.e = engine

    def __call__(self, leaf_state, leaf_mask, leaf_valid):
        B = leaf_state.shape[0]
        pi = torch.empty((B, ACTIONS), dtype=torch.float32, device=self.e.device)
        v = torch.empty((B, self.e.n), dtype=torch.float32, device=self.e.device)
        _lib.check(self.e.L.spl_hash_eval(self.e.ctx, B, _ptr(leaf_state), _ptr(leaf_mask), _ptr(pi),
                                          _ptr(v), self.e._s()), "spl_hash_eval")
        return pi, v


class BatchedMCTS:
    def __init__(self, engine, B, args=None, evaluator=None, dirichlet_noise=False, seed=0x5EED,
                 board_base=0, node_cap=None, edge_cap=None, selfplay=False, node_boards=None):
        self.e = engine
        self.L = engine.L
        self.B = B
        self.args = args
        sims = int(_arg(args, "numMCTSSims"))
        cfg = _lib.MctsConfig()
        cfg.num_sims = sims
        cfg.ratio_full = int(_arg(args, "ratio_fullMCTS"))
        cfg.prob_full = float(_arg(args, "prob_fullMCTS"))
        cfg.cpuct = float(_arg(args, "cpuct"))
        cfg.fpu = float(_arg(args, "fpu"))
        cfg.forced_playouts = int(bool(_arg(args, "forced_playouts")))
        cfg.dirichlet_alpha = float(_arg(args, "dirichletAlpha")) if dirichlet_noise else 0.0
        cfg.dirichlet_temp = float(_arg(args, "temperature")[0])
        cfg.temp_threshold = int(_arg(args, "tempThreshold"))
        cfg.seed = seed
        cfg.board_base = board_base
        cfg.selfplay = int(bool(selfplay))
        cfg.out_cap = int(getattr(self, "_selfplay_out_cap", 0))
        cfg.node_boards = 1 if node_boards is None else int(bool(node_boards))
        cfg.node_cap, cfg.edge_cap = self._caps(engine, B, sims, cfg, node_cap, edge_cap, node_boards is None)
        self.cfg = cfg
        h = C.c_void_p()
        _lib.check(self.L.spl_mcts_create(engine.ctx, B, C.byref(cfg), C.byref(h)), "spl_mcts_create")
        self.h = h
        dev = engine.device
        self.leaf_state = engine.new_state(B)
        self.leaf_mask = torch.zeros((B, MASK_WORDS), dtype=torch.int64, device=dev)
        self.leaf_valid = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.evaluator = evaluator or HashEvaluator(engine)
        self._hdr = torch.empty((B, HDR_DTYPE.itemsize // 4), dtype=torch.int32, device=dev)

    MEM_FRACTION = 0.8     # of the device's free memory a default-sized arena may take

    def _caps(self, engine, B, sims, cfg, node_cap, edge_cap, auto_boards=False):
        """Per-tree pool sizes. A search adds at most `sims` nodes, but the
        kept table (every node whose round exceeds the root's, MCTS.py semantics) keeps
        growing through a game: at genbu's arguments and 100 simulations, steady-state
        trees reach ~1,850 nodes / 50 K edges (tools/tree_sizes.py, 15-19 edges per node on
        average). Default: 16 x sims + 256 node slots, 32 edges per slot (garbage is only
        collected when a search would not fit, so the slots also hold dead nodes); when B
        such trees do not fit MEM_FRACTION of the free HBM, 24 edges per slot and as many
        slots as fit (searches then start on pruned trees under pressure, counted in the
        tree headers). Node boards (cfg.node_boards, a speed option) are kept unless the
        caller chose (auto_boards False); under memory pressure they are dropped first, so
        capacity (the reference's exact table) wins over descent speed."""
        if node_cap and edge_cap:
            return int(node_cap), int(edge_cap)
        nc = int(node_cap or 16 * sims + 256)
        ec = int(edge_cap or 32 * nc)

        def plan(nc_, ec_):
            cfg.node_cap, cfg.edge_cap = int(nc_), int(ec_)
            return int(self.L.spl_mcts_plan_bytes(engine.ctx, B, C.byref(cfg)))
        if engine.device.type != "cuda" or (node_cap or edge_cap):
            return nc, ec
        free = torch.cuda.mem_get_info(engine.device)[0]
        limit = int(self.MEM_FRACTION * free)
        if plan(nc, ec) <= limit:
            return nc, ec
        if auto_boards and cfg.node_boards:
            cfg.node_boards = 0
            if plan(nc, ec) <= limit:
                return nc, ec
        ratio = 24
        lo = plan(64, 64 * ratio)
        per = (plan(1064, 1064 * ratio) - lo) / 1000.0
        nc = max(64, int((limit - lo) / per) + 64)
        while nc > 64 and plan(nc, nc * ratio) > limit:
            nc = int(nc * 0.97)
        return nc, nc * ratio

    def __del__(self):
        if getattr(self, "h", None) is not None:
            self.L.spl_mcts_destroy(self.h)
            self.h = None

    @property
    def device_bytes(self):
        return int(self.L.spl_mcts_device_bytes(self.h))

    def capacity_events(self, hdr=None):
        """Trees pruned / emptied at a search start and simulations whose leaf did not fit
        (0 everywhere = every search ran on the reference's exact table)."""
        h = self.headers() if hdr is None else hdr
        return {"prunes": int(h["prunes"].sum()), "resets": int(h["resets"].sum()),
                "unexpanded": int(h["unexpanded"].sum())}

    # ---------------------------------------------------------------- primitives
    def set_roots(self, roots, keep_tree=True, force_full=True):
        _lib.check(self.L.spl_mcts_set_roots(self.h, _ptr(roots), int(keep_tree), int(force_full),
                                             self.e._s()), "spl_mcts_set_roots")

    def set_roots_active(self, roots, active, keep_tree=True, force_full=True):
        """set_roots for the trees with active[t] != 0 (uint8 [B], device); the others keep
        their tree and run no simulations until re-rooted."""
        _lib.check(self.L.spl_mcts_set_roots_active(self.h, _ptr(roots), _ptr(active), int(keep_tree),
                                                    int(force_full), self.e._s()),
                   "spl_mcts_set_roots_active")

    def pick_best(self, active=None, board_base=0, stream=0, out=None):
        """getActionProb(temp=0) + argmax (MCTS.py:87-92) for the active trees -> int16 [B]
        (entries of inactive trees untouched); ties by Philox (seed, board_base + t, stream)."""
        out = out if out is not None else torch.full((self.B,), -1, dtype=torch.int16, device=self.e.device)
        _lib.check(self.L.spl_mcts_pick_best(self.h, _ptr(active), int(board_base), int(stream), _ptr(out),
                                             self.e._s()), "spl_mcts_pick_best")
        return out

    def search(self):
        """Run simulations until every tree has spent its budget."""
        for _ in range(int(self.headers()["budget"].max())):
            self.simulate()

    def simulate(self):
        """One simulation on every tree with budget left: select -> evaluate -> backup."""
        s = self.e._s()
        _lib.check(self.L.spl_mcts_select(self.h, _ptr(self.leaf_state), _ptr(self.leaf_mask),
                                          _ptr(self.leaf_valid), s), "spl_mcts_select")
        pi, v = self.evaluator(self.leaf_state, self.leaf_mask, self.leaf_valid)
        _lib.check(self.L.spl_mcts_backup(self.h, _ptr(self.leaf_mask), _ptr(pi), _ptr(v), s),
                   "spl_mcts_backup")

    def headers(self):
        _lib.check(self.L.spl_mcts_headers(self.h, _ptr(self._hdr), self.e._s()), "spl_mcts_headers")
        return self._hdr.cpu().numpy().view(HDR_DTYPE).reshape(self.B)

    def tree_sizes(self):
        """int32 [B, 4] per tree: node slots used, edge slots used, live nodes (root + rounds
        beyond the root's: what GC keeps), live edges."""
        out = torch.empty((self.B, 4), dtype=torch.int32, device=self.e.device)
        _lib.check(self.L.spl_mcts_tree_sizes(self.h, _ptr(out), self.e._s()), "spl_mcts_tree_sizes")
        return out.cpu().numpy()

    def root_stats(self, adjusted=False):
        B, dev = self.B, self.e.device
        counts = torch.empty((B, ACTIONS), dtype=torch.int64, device=dev)
        qsa = torch.empty((B, ACTIONS), dtype=torch.float64, device=dev)
        probs = torch.empty((B, ACTIONS), dtype=torch.float64, device=dev)
        q = torch.empty((B, self.e.n), dtype=torch.float64, device=dev)
        adj = torch.empty((B, ACTIONS), dtype=torch.int64, device=dev) if adjusted else None
        _lib.check(self.L.spl_mcts_root_stats(self.h, _ptr(counts), _ptr(qsa), _ptr(probs), _ptr(q),
                                              _ptr(adj), self.e._s()), "spl_mcts_root_stats")
        return (counts, qsa, probs, q, adj) if adjusted else (counts, qsa, probs, q)

    def root_priors(self):
        """Stored root priors Ps (float32 [B,409]; MCTS.nodes_data[s][2], noised when root
        Dirichlet noise was applied)."""
        ps = torch.empty((self.B, ACTIONS), dtype=torch.float32, device=self.e.device)
        _lib.check(self.L.spl_mcts_root_priors(self.h, _ptr(ps), self.e._s()), "spl_mcts_root_priors")
        return ps

    # ---------------------------------------------------------------- reference API
    def get_action_prob(self, canonical_boards, force_full_search=True, keep_tree=True):
        """Batched MCTS.getActionProb(temp=1) (MCTS.py:45-97): returns (probs f64 [B,409],
        q f64 [B,n], is_full_search bool [B], counts i64 [B,409])."""
        keep_tree = keep_tree and not getattr(self, "_reset_pending", False)
        self._reset_pending = False
        self.set_roots(canonical_boards, keep_tree=keep_tree, force_full=force_full_search)
        hdr = self.headers()
        for _ in range(int(hdr["budget"].max())):
            self.simulate()
        hdr = self.headers()
        if hdr["overflow"].any():
            raise _lib.EngineError(f"tree capacity exceeded on {int((hdr['overflow'] != 0).sum())} trees")
        counts, _, probs, q = self.root_stats()
        return probs, q, torch.from_numpy(hdr["full"] != 0), counts

    def reset(self):
        """reset_all_search_trees (MCTS.py:188-192): next set_roots starts empty trees."""
        self._reset_pending = True
