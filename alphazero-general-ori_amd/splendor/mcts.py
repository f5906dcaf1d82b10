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
import os

import numpy as np
import torch

from . import _lib
from .env import ACTIONS, MASK_WORDS, _ptr

# TreeHdr (csrc/mcts_device.h), 208 bytes
HDR_DTYPE = np.dtype([
    ("node_count", "<i4"), ("edge_count", "<i4"), ("root", "<i4"), ("sims_done", "<i4"),
    ("budget", "<i4"), ("full", "<i4"), ("noise_pending", "<i4"), ("depth", "<i4"),
    ("leaf_kind", "<i4"), ("player", "<i4"), ("episode_step", "<i4"), ("move_no", "<i4"),
    ("game_no", "<i4"), ("overflow", "<i4"), ("n_examples", "<i4"), ("leaf_round", "<i4"),
    ("leaf_k0", "<u8"), ("leaf_k1", "<u8"), ("leaf_v", "<f4", (4,)),
    ("games_done", "<i4"), ("forced", "<i4"), ("moves", "<i4"), ("wd_search", "<i4"),
    ("prunes", "<i4"), ("resets", "<i4"), ("unexpanded", "<i4"), ("gc_state", "<i4"),
    ("units_gc", "<i8"), ("enext", "<i8"),
    ("npg", "<i4"), ("epg", "<i4"), ("eleft", "<i4"), ("live_gc", "<i4"),
    ("root_round", "<i4"), ("gc_queued", "<i4"), ("withdrawals", "<i4"), ("gcs", "<i4"),
    ("leaf_hslot", "<i4"), ("leaf_slot", "<i4"), ("depth_max", "<i4"), ("depth_sum", "<i4"),
    ("resume", "<i4"), ("sims_backed", "<i4"), ("exact_wide", "<i4"), ("big_moves", "<i4")])
assert HDR_DTYPE.itemsize == 208

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
    """Deterministic stand-in network (spl_hash_eval_mode); identical to the oracle's
    or_fake_predict. mode 0: spread priors and values (shallow trees); mode 1: peaked priors
    and values near +-1, like the random-init SplendorNNet (the bench's deep trees)."""

    def __init__(self, engine, mode=0):
        self.e = engine
        self.mode = int(mode)

    def __call__(self, leaf_state, leaf_mask, leaf_valid):
        B = leaf_state.shape[0]
        pi = torch.empty((B, ACTIONS), dtype=torch.float32, device=self.e.device)
        v = torch.empty((B, self.e.n), dtype=torch.float32, device=self.e.device)
        _lib.check(self.e.L.spl_hash_eval_mode(self.e.ctx, B, _ptr(leaf_state), _ptr(leaf_mask), _ptr(pi),
                                               _ptr(v), self.mode, self.e._s()), "spl_hash_eval_mode")
        return pi, v


class BatchedMCTS:
    def __init__(self, engine, B, args=None, evaluator=None, dirichlet_noise=False, seed=0x5EED,
                 board_base=0, node_cap=None, edge_cap=None, selfplay=False, node_boards=None,
                 pool_nodes=None, pool_edges=None, mem_budget=None):
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
        self._plan(engine, B, sims, cfg, node_cap, edge_cap, pool_nodes, pool_edges, node_boards is None,
                   mem_budget)
        self.cfg = cfg
        h = C.c_void_p()
        _lib.check(self.L.spl_mcts_create(engine.ctx, B, C.byref(cfg), C.byref(h)), "spl_mcts_create")
        self.h = h
        dev = engine.device
        self.leaf_state = engine.new_state(B)
        self.leaf_mask = torch.zeros((B, MASK_WORDS), dtype=torch.int64, device=dev)
        self.leaf_valid = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.leaf_index = torch.zeros(B, dtype=torch.int32, device=dev)
        self.leaf_count = torch.zeros((B + 63) // 64, dtype=torch.int32, device=dev)   # per 64-tree segment
        self.evaluator = evaluator or HashEvaluator(engine)
        self._hdr = torch.empty((B, HDR_DTYPE.itemsize // 4), dtype=torch.int32, device=dev)

    MEM_FRACTION = 0.8      # of the device's free memory a default-sized arena may take
    UNITS_PER_NODE = 20     # pool edge-unit : node-slot ratio (8-byte units: one per edge, three per
                            # edge with statistics; live trees ~16 edges + ~4 units of visit records
                            # per node, profiles/r04_tree_sizes_*); node slots are ~85 B, so erring
                            # towards nodes is cheap
    NODE_MAX = 45056        # per-tree node maximum (transposition table 64 K slots at most)

    @staticmethod
    def default_node_cap(sims):
        """Per-tree node maximum: live self-play trees reach ~18 x sims nodes at 100
        simulations and ~22 x sims at 1,600 (profiles/r03_tree_sizes_*: max 1,845 / 35,407);
        lazy collection lets a tree hold up to twice its live size, so 64 x sims + 4,096,
        at most NODE_MAX."""
        return min(64 * sims + 4096, BatchedMCTS.NODE_MAX)

    def _plan(self, engine, B, sims, cfg, node_cap, edge_cap, pool_nodes, pool_edges, auto_boards, mem_budget):
        """Tree maxima and the shared pools. node_cap / edge_cap: the largest
        single tree (transposition table, page tables; edge_cap in 8-byte edge units);
        pool_nodes / pool_edges: node slots and edge units shared by all B trees. Explicit caps
        without pools keep the static layout (pool = B x cap). Default: pools fill
        MEM_FRACTION of the free HBM (or mem_budget bytes) at UNITS_PER_NODE units per node
        slot; node boards (a speed option) are kept when the pools then still hold 8 x sims +
        512 node slots per tree, else dropped first: capacity (the reference's exact table)
        wins over descent speed."""
        nc = int(node_cap or self.default_node_cap(sims))
        ec = int(edge_cap or 32 * nc)
        cfg.node_cap, cfg.edge_cap = nc, ec
        cfg.pool_nodes, cfg.pool_edges = int(pool_nodes or 0), int(pool_edges or 0)
        if (node_cap or edge_cap) and not (pool_nodes or pool_edges):
            return                                          # static: B x caps
        if pool_nodes and pool_edges:
            return
        if engine.device.type != "cuda":
            cfg.pool_nodes = cfg.pool_nodes or B * nc
            cfg.pool_edges = cfg.pool_edges or B * ec
            return
        budget = int(mem_budget) if mem_budget else int(self.MEM_FRACTION * torch.cuda.mem_get_info(engine.device)[0])
        R = self.UNITS_PER_NODE

        def plan(pn):
            cfg.pool_nodes, cfg.pool_edges = int(pn), int(pn) * R
            return int(self.L.spl_mcts_plan_bytes(engine.ctx, B, C.byref(cfg)))

        def fit():
            lo = plan(B * 64)
            per = (plan(B * 64 + (1 << 20)) - lo) / float(1 << 20)
            return max(B * 64, int((budget - lo) / per) + B * 64 - 4096)
        pn = fit()
        if auto_boards and cfg.node_boards and pn < B * (8 * sims + 512):
            cfg.node_boards = 0
            pn = fit()
        while pn > B * 64 and plan(pn) > budget:
            pn = int(pn * 0.98)
        cfg.pool_nodes, cfg.pool_edges = int(pool_nodes or pn), int(pool_edges or pn * R)

    def pool_state(self):
        """(free node pages, free edge pages, failed node-page requests, failed edge-page
        requests) of the shared pools, and their sizes in pages."""
        out = torch.empty(4, dtype=torch.int32, device=self.e.device)
        _lib.check(self.L.spl_mcts_pool_state(self.h, _ptr(out), self.e._s()), "spl_mcts_pool_state")
        pages = (C.c_longlong * 4)()
        _lib.check(self.L.spl_mcts_pool_pages(self.h, pages), "spl_mcts_pool_pages")
        f = out.tolist()
        return {"free_node_pages": f[0], "free_edge_pages": f[1], "node_page_misses": f[2],
                "edge_page_misses": f[3], "node_pages": int(pages[0]), "edge_pages": int(pages[1]),
                "nodes_per_page": int(pages[2]), "units_per_page": int(pages[3])}

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

    def check_capacity(self, allow=False, hdr=None):
        """Raise EngineError on any capacity event (a search that deviated from the
        reference's table) unless allow; returns the events."""
        ev = self.capacity_events(hdr)
        if not allow and any(ev.values()):
            raise _lib.EngineError(f"capacity events {ev}: searches deviated from the reference table "
                                   f"(raise node_cap / pool sizes)")
        return ev

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

    # terminal leaves backed up on a side stream during the network (SPLENDOR_OVERLAP=1: on; measured slower: the backup waves delay the network workgroups)
    OVERLAP_TERMINAL = os.environ.get("SPLENDOR_OVERLAP", "0") != "0"

    def simulate(self, defer_gc=False):
        """One simulation on every tree with budget left: select -> evaluate -> backup. An
        evaluator that can take a compacted leaf list (`indexed`, the fused network) runs on
        the trees whose leaf needs the network only; the trees whose leaf is terminal are
        backed up meanwhile on a side stream (trees are independent; spl_mcts_backup_kind).
        defer_gc (self-play): the caller commits before the next select, and that commit's
        collection takes the withdrawn simulations' trees (SPL_BACKUP_DEFER_GC)."""
        s = self.e._s()
        dg = _lib.BACKUP_DEFER_GC if defer_gc else 0
        if getattr(self.evaluator, "indexed", False):
            _lib.check(self.L.spl_mcts_select_compact(self.h, _ptr(self.leaf_state), _ptr(self.leaf_mask),
                                                      _ptr(self.leaf_valid), _ptr(self.leaf_index),
                                                      _ptr(self.leaf_count), s), "spl_mcts_select_compact")
            if self.OVERLAP_TERMINAL and self.e.device.type == "cuda":
                cur = torch.cuda.current_stream(self.e.device)
                side = getattr(self, "_side", None)
                if side is None:
                    side = self._side = torch.cuda.Stream(device=self.e.device)
                side.wait_stream(cur)
                _lib.check(self.L.spl_mcts_backup_kind(self.h, None, None, None, 2, C.c_void_p(side.cuda_stream)),
                           "spl_mcts_backup_kind")
                pi, v = self.evaluator(self.leaf_state, self.leaf_mask, self.leaf_valid, index=self.leaf_index,
                                       count=self.leaf_count)
                cur.wait_stream(side)
                _lib.check(self.L.spl_mcts_backup_kind(self.h, _ptr(self.leaf_mask), _ptr(pi), _ptr(v), 1 | dg, s),
                           "spl_mcts_backup_kind")
                return
            pi, v = self.evaluator(self.leaf_state, self.leaf_mask, self.leaf_valid, index=self.leaf_index,
                                   count=self.leaf_count)
        else:
            _lib.check(self.L.spl_mcts_select(self.h, _ptr(self.leaf_state), _ptr(self.leaf_mask),
                                              _ptr(self.leaf_valid), s), "spl_mcts_select")
            pi, v = self.evaluator(self.leaf_state, self.leaf_mask, self.leaf_valid)
        _lib.check(self.L.spl_mcts_backup_kind(self.h, _ptr(self.leaf_mask), _ptr(pi), _ptr(v), 3 | dg, s),
                   "spl_mcts_backup_kind")

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
        ev = self.capacity_events(hdr)
        if any(ev.values()) and not getattr(self, "_warned_capacity", False):
            import warnings
            warnings.warn(f"BatchedMCTS capacity events {ev}: some searches ran on pruned trees or "
                          f"left leaves unstored (raise node_cap / the pools)")
            self._warned_capacity = True
        counts, _, probs, q = self.root_stats()
        return probs, q, torch.from_numpy(hdr["full"] != 0), counts

    def reset(self):
        """reset_all_search_trees (MCTS.py:188-192): next set_roots starts empty trees."""
        self._reset_pending = True
