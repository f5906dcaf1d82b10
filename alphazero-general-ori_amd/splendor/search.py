"""The reference's MCTS plug-in API (MCTS.py:16-192) over the device-resident tree.

    MCTS(game, nnet, args, dirichlet_noise=False).getActionProb(canonicalBoard, temp=1,
                                                                force_full_search=False)
    -> (probs list[409], q list[n], is_full_search)
    MCTS.reset_all_search_trees()

One persistent device tree per MCTS object (the reference's transposition table persists
across moves until reset_all_search_trees, MCTS.py:188-192). The network is queried through
`nnet.predict(board, valid_actions)` exactly as the reference does (batch 1, host round
trip), unless `nnet` is a splendor.NNet.NNetWrapper, whose SplendorNNet then runs on the
device next to the tree with no host round trip.
"""
import weakref

import numpy as np
import torch

from .env import ACTIONS, unpack_mask
from .mcts import BatchedMCTS


class PredictEvaluator:
    """Leaf evaluation through a reference-style `nnet.predict(board, valids)`."""

    def __init__(self, engine, nnet):
        self.e, self.nnet = engine, nnet

    def __call__(self, leaf_state, leaf_mask, leaf_valid):
        B, n, dev = leaf_state.shape[0], self.e.n, self.e.device
        pi = np.zeros((B, ACTIONS), np.float32)
        v = np.zeros((B, n), np.float32)
        need = leaf_valid.cpu().numpy().astype(bool)
        if need.any():
            boards = leaf_state.cpu().numpy()
            masks = unpack_mask(leaf_mask).cpu().numpy()
            for b in np.flatnonzero(need):
                p, val = self.nnet.predict(boards[b], masks[b])
                pi[b] = np.asarray(p, np.float32)
                v[b] = np.asarray(val, np.float32)
        return torch.from_numpy(pi).to(dev), torch.from_numpy(v).to(dev)


def evaluator_for(engine, nnet, batch=1):
    from .NNet import NNetWrapper
    from .nnet import LeafEvaluator
    if isinstance(nnet, NNetWrapper):
        return LeafEvaluator(engine, nnet.nnet, batch, use_graph=False)
    return PredictEvaluator(engine, nnet)


class MCTS:
    _instances = weakref.WeakSet()

    def __init__(self, game, nnet, args, dirichlet_noise=False, batch_info=None):
        self.game, self.nnet, self.args = game, nnet, args
        seed = getattr(args, "seed", None) if not isinstance(args, dict) else args.get("seed")
        self._tree = BatchedMCTS(game.engine, 1, args, evaluator_for(game.engine, nnet),
                                 dirichlet_noise=dirichlet_noise, seed=seed or 0x5EED)
        self._fresh = True
        MCTS._instances.add(self)

    def getActionProb(self, canonicalBoard, temp=1, force_full_search=False, bias=None):
        dev = self.game.engine.device
        root = torch.from_numpy(np.ascontiguousarray(canonicalBoard, dtype=np.int8)[None]).to(dev)
        self._tree.set_roots(root, keep_tree=not self._fresh, force_full=force_full_search)
        self._fresh = False
        hdr = self._tree.headers()
        for _ in range(int(hdr["budget"][0])):
            self._tree.simulate()
        hdr = self._tree.headers()
        if hdr["overflow"][0]:
            raise RuntimeError("search tree capacity exceeded (raise node_cap / edge_cap)")
        _, _, _, q, adj = self._tree.root_stats(adjusted=True)
        counts = adj[0].cpu().numpy()
        q = [float(x) for x in q[0].cpu().numpy()]
        full = bool(hdr["full"][0])
        if temp == 0:                                          # MCTS.py:87-92
            best = np.flatnonzero(counts == counts.max())
            probs = [0] * len(counts)
            probs[int(np.random.choice(best))] = 1
            return probs, q, full
        x = [float(c) ** (1.0 / temp) for c in counts]          # MCTS.py:94-97
        s = float(sum(x))
        return [c / s for c in x], q, full

    @staticmethod
    def reset_all_search_trees():
        for m in list(MCTS._instances):
            m._fresh = True
