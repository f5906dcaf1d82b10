"""Batched self-play: Coach.executeEpisode (Coach.py:50-100) for B concurrent games.

Every iteration runs one MCTS simulation on every game's tree (select -> leaf network ->
backup) and then `spl_mcts_commit`, which plays the move of every game whose search budget
is spent (policy, example, temperature sampling, chance step, end of game, re-root). Games
restart automatically, so all B trees stay busy; moves commit asynchronously per game
(full/fast search budgets differ, MCTS.py:54-55). The whole iteration is a fixed sequence
of stream-ordered launches, captured once into a HIP graph and replayed.

Finished examples are (board, pi, winner, scdiff, valids, surprise) as assembled at
Coach.py:91-98, drained as device tensors (`drain()`), optionally gathered across ranks
(`gather_examples`, RCCL all-gather) and expanded with `symmetries`.
"""
import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from .env import ACTIONS, MASK_WORDS, _ptr
from .mcts import BatchedMCTS


class SelfPlay(BatchedMCTS):
    """out_cap: finished-example queue (default: one full game of examples per tree, B x
    (62n + 2), so a drain per game length cannot overflow it; examples that still do not fit
    are counted and `drain` raises)."""

    def __init__(self, engine, B, args=None, evaluator=None, dirichlet_noise=True, seed=0x5EED,
                 board_base=0, out_cap=None, node_cap=None, edge_cap=None, node_boards=None,
                 pool_nodes=None, pool_edges=None, mem_budget=None):
        self._selfplay_out_cap = int(out_cap or B * (62 * engine.n + 2))
        self._dropped_seen = 0
        super().__init__(engine, B, args, evaluator, dirichlet_noise=dirichlet_noise, seed=seed,
                         board_base=board_base, node_cap=node_cap, edge_cap=edge_cap, selfplay=True,
                         node_boards=node_boards, pool_nodes=pool_nodes, pool_edges=pool_edges,
                         mem_budget=mem_budget)
        self.graph = None
        self.graph_k = None

    GRAPH_ITERS = 8

    def run(self, k, use_graph=True):
        """k iterations. With use_graph, replays of a graph of GRAPH_ITERS iterations (a graph
        launch leaves ~9 us of idle GPU before the next one, measured; one per 8 iterations
        instead of one per iteration), single-iteration replays for the remainder."""
        if not use_graph:
            for _ in range(k):
                self._iteration()
            return
        done = 0
        if self.graph is None:
            self.step(use_graph=True)                # eager warm-up iteration + 1-iteration graph
            done = 1
        n, r = divmod(k - done, self.GRAPH_ITERS)
        if n and self.graph_k is None:
            self.graph_k = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_k):     # capture only; nothing executes
                for _ in range(self.GRAPH_ITERS):
                    self._iteration()
        for _ in range(n):
            self.graph_k.replay()
        for _ in range(r):
            self.graph.replay()

    def reset(self):
        _lib.check(self.L.spl_mcts_reset_games(self.h, self.e._s()), "spl_mcts_reset_games")

    def restart(self, games):
        """Abandon the current game of every tree with games[t] (B bools, or a list of tree
        ids) and deal its next one; staged examples of the abandoned games are discarded.
        Between iterations only. bench.py uses it to spread games that were dealt together
        over the phases of a game (its `--stagger` warm-up)."""
        if not (torch.is_tensor(games) and games.dtype == torch.bool):
            ids = torch.as_tensor(games, dtype=torch.long)
            games = torch.zeros(self.B, dtype=torch.bool)
            games[ids] = True
        mask = games.to(device=self.e.device, dtype=torch.uint8).contiguous()
        if mask.numel() != self.B:
            raise ValueError(f"restart mask of {mask.numel()} entries for {self.B} games")
        _lib.check(self.L.spl_mcts_restart_games(self.h, _ptr(mask), self.e._s()), "spl_mcts_restart_games")
        self._keep = mask                        # alive until the stream has used it

    # the backup leaves the withdrawn simulations' trees to the commit's collection
    # (SPL_BACKUP_DEFER_GC; SPLENDOR_DEFER_GC=0: collect after the backup as well)
    DEFER_GC = os.environ.get("SPLENDOR_DEFER_GC", "1") != "0"

    def _iteration(self):
        self.simulate(defer_gc=self.DEFER_GC)
        _lib.check(self.L.spl_mcts_commit(self.h, self.e._s()), "spl_mcts_commit")

    def step(self, use_graph=False):
        if not use_graph:
            self._iteration()
            return
        if self.graph is None:
            if hasattr(self.evaluator, "use_graph"):
                self.evaluator.use_graph = False     # the whole iteration is one graph
            self._iteration()                        # eager iteration: warms libraries
            torch.cuda.synchronize(self.e.device)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):       # capture only; nothing executes
                self._iteration()
            return
        self.graph.replay()

    def counters(self):
        """(examples queued, examples dropped so far) — one small device read."""
        c = torch.empty(2, dtype=torch.int32, device=self.e.device)
        _lib.check(self.L.spl_mcts_counters(self.h, _ptr(c), self.e._s()), "spl_mcts_counters")
        q, d = c.tolist()
        return q, d

    def dropped_examples(self):
        return self.counters()[1]

    def drain(self, allow_drops=False):
        """Move finished examples out of the device queue: dict of device tensors. Raises
        EngineError if examples were lost to a full queue since the last drain (training
        data must not vanish silently) unless allow_drops."""
        queued, dropped = self.counters()
        if dropped > self._dropped_seen and not allow_drops:
            lost = dropped - self._dropped_seen
            self._dropped_seen = dropped
            raise _lib.EngineError(f"{lost} finished examples dropped: the example queue (out_cap="
                                   f"{self._selfplay_out_cap}) filled up between drains")
        self._dropped_seen = dropped
        E, n, dev = min(queued, self._selfplay_out_cap), self.e.n, self.e.device
        out = {
            "board": torch.empty((E, self.e.rows, 7), dtype=torch.int8, device=dev),
            "pi": torch.empty((E, ACTIONS), dtype=torch.float32, device=dev),
            "valids": torch.empty((E, MASK_WORDS), dtype=torch.int64, device=dev),
            "winner": torch.empty((E, n), dtype=torch.float32, device=dev),
            "scdiff": torch.empty((E, n), dtype=torch.int32, device=dev),
            "surprise": torch.empty((E, n), dtype=torch.float32, device=dev),
            "meta": torch.empty((E, 4), dtype=torch.int32, device=dev),
        }
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(self.L.spl_mcts_drain_examples(
            self.h, _ptr(out["board"]), _ptr(out["pi"]), _ptr(out["valids"]), _ptr(out["winner"]),
            _ptr(out["scdiff"]), _ptr(out["surprise"]), _ptr(out["meta"]), E, _ptr(cnt), self.e._s()),
            "drain")
        k = int(cnt.item())
        return {key: v[:k] for key, v in out.items()}

    def stats(self):
        h = self.headers()
        return {"games_done": int(h["games_done"].sum()), "moves": int(h["moves"].sum()),
                "withdrawals": int(h["withdrawals"].sum()), "collections": int(h["gcs"].sum()),
                "overflow": int((h["overflow"] != 0).sum()),
                "nodes_max": int(h["node_count"].max()), "edges_max": int(h["edge_count"].max()),
                "leaf_depth_now": float(h["depth"].mean()), "leaf_depth_max": int(h["depth"].max()),
                "depth_sum": int(h["depth_sum"].astype("int64").sum()), "depth_max_all": int(h["depth_max"].max()),
                "sims_backed": int(h["sims_backed"].astype("int64").sum()),
                "exact_wide": int(h["exact_wide"].astype("int64").sum()),
                "big_moves": int(h["big_moves"].astype("int64").sum()),
                **self.capacity_events(h), "examples_dropped": self.dropped_examples()}

    # per-tree cumulative 32-bit header counters (depth_sum wraps after ~40 M simulations of a
    # long-lived tree at depth ~50); window deltas are taken per tree modulo 2^32, then summed
    COUNTERS = {"games_done": "games_done", "moves": "moves", "withdrawals": "withdrawals",
                "collections": "gcs", "depth_sum": "depth_sum", "sims_backed": "sims_backed",
                "exact_wide": "exact_wide", "big_moves": "big_moves", "prunes": "prunes", "resets": "resets",
                "unexpanded": "unexpanded"}

    def counter_snapshot(self):
        h = self.headers()
        return {k: h[f].astype(np.uint32) for k, f in self.COUNTERS.items()}

    @staticmethod
    def counter_delta(before, after):
        """Window totals of counter_snapshot()s: wrap-safe as long as no single tree's counter
        advances by 2^32 or more inside the window."""
        return {k: int((after[k] - before[k]).astype(np.int64).sum()) for k in before}


def pack_examples(examples):
    """Columns -> one fixed-size byte record per example ([E, bytes] uint8), in key order;
    returns (records, layout) for unpack_examples."""
    E = next(iter(examples.values())).shape[0]
    cols, layout = [], []
    for key, t in examples.items():
        row = 1
        for d in t.shape[1:]:
            row *= int(d)
        b = t.contiguous().reshape(E, row).view(torch.uint8)
        cols.append(b)
        layout.append((key, t.dtype, tuple(t.shape[1:]), b.shape[1]))
    return torch.cat(cols, 1), layout


def unpack_examples(records, layout):
    out, off = {}, 0
    E = records.shape[0]
    for key, dtype, shape, nb in layout:
        col = torch.empty((E, nb), dtype=torch.uint8, device=records.device)
        col.copy_(records[:, off:off + nb])
        out[key] = col.view(dtype).reshape((E,) + shape)
        off += nb
    return out


def gather_examples(examples, group=None):
    """Episode-end exchange across ranks (torch.distributed, RCCL on
    ROCm): every example packed into one fixed-size byte record (board, pi, valids, winner,
    scdiff, surprise, meta), then one all_gather of the counts and one all_gather of the
    records padded to the largest shard; rank order and per-rank example order preserved.
    Under the gloo backend device tensors travel through host memory."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return examples
    world = dist.get_world_size(group)
    rec, layout = pack_examples(examples)
    dev = rec.device
    if dist.get_backend(group) == "gloo" and dev.type == "cuda":
        rec = rec.cpu()
    k = torch.tensor([rec.shape[0]], dtype=torch.int64, device=rec.device)
    sizes = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(sizes, k, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx, rec.shape[1]), dtype=torch.uint8, device=rec.device)
    pad[:rec.shape[0]] = rec
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    allrec = torch.cat([p[:s] for p, s in zip(parts, sizes)]).to(dev)
    return unpack_examples(allrec, layout)


def broadcast_network(net, src=0, group=None):
    """Weights of rank `src` to every rank (one broadcast of the
    SplendorNNet parameters and BatchNorm statistics, repeated only when the network
    changes), flattened into one buffer so it is a single collective."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return net
    tensors = [t for t in net.state_dict().values() if t.is_floating_point()]
    flat = torch.cat([t.detach().reshape(-1).float() for t in tensors])
    dist.broadcast(flat, src=src, group=group)
    off = 0
    with torch.no_grad():
        for t in tensors:
            t.copy_(flat[off:off + t.numel()].view_as(t).to(t.dtype))
            off += t.numel()
    return net
