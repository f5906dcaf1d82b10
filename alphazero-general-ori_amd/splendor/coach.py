"""Coach plug-in: Coach.executeEpisode (Coach.py:50-100) for many games at once.

`Coach(game, nnet, args, batch=B).executeEpisodes(k)` plays self-play games on B device
trees concurrently (splendor.selfplay.SelfPlay) until k games have finished, expands every
recorded position with getSymmetries (Coach.py:77-80, device kernel spl_symmetries) and
returns the reference's example records (board, pi, winner, scdiff, valids, surprise)
(Coach.py:91-98). `executeEpisode()` is the one-game form. `executeIteration(k)` returns
the same examples as a columnar `ExampleSet` and appends it to `trainExamplesHistory`
(an `ExampleHistory`, saved as .npz by `saveTrainExamples`, Coach.py:167-190). `learn()`
is Coach.learn (Coach.py:102-164): self-play iterations, training on the example history,
the new-vs-previous BatchedArena gate and checkpoints.
"""
import numpy as np
import torch

from .env import unpack_mask
from .arena import BatchedArena, accept_new_network
from .examples import ExampleHistory, ExampleSet
from .search import evaluator_for
from .selfplay import SelfPlay, gather_examples


def _arg(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


def expand_symmetries(engine, ex):
    """Apply Board.get_symmetries to drained examples (device tensors, reference order);
    winner / scdiff / surprise are shared by all variants of a position."""
    if ex["board"].shape[0] == 0:
        return ex
    s, p, v, present = engine.symmetries(ex["board"], ex["pi"], ex["valids"])
    keep = present.bool()
    idx = torch.arange(ex["board"].shape[0], device=keep.device).unsqueeze(1).expand_as(keep)[keep]
    out = {"board": s[keep], "pi": p[keep], "valids": v[keep]}
    for k in ("winner", "scdiff", "surprise"):
        out[k] = ex[k][idx]
    return out


class Coach:
    def __init__(self, game, nnet, args, batch=None, seed=0x5EED, board_base=0):
        self.game, self.nnet, self.args = game, nnet, args
        B = int(batch or _arg(args, "numEps", 1))
        self.B = B
        self.seed = seed
        self.sp = SelfPlay(game.engine, B, args, evaluator=evaluator_for(game.engine, nnet, B),
                           dirichlet_noise=float(_arg(args, "dirichletAlpha", 0.0)) > 0, seed=seed,
                           board_base=board_base)
        self.sp.reset()
        self.trainExamplesHistory = ExampleHistory(_arg(args, "numItersHistory"))

    def run_iterations(self, k, use_graph=False):
        self.sp.run(k, use_graph=use_graph)

    def executeEpisodes(self, num_games, with_symmetries=True, as_tuples=True, gather=False):
        """Play until num_games games have finished (counted from the call), draining the
        example queue every 32 iterations. Raises EngineError if a tree froze (search path
        overflow) or finished examples were dropped. Capacity events (trees pruned under
        memory pressure) are counted in self.sp.stats()."""
        from . import _lib
        collected, done = [], 0
        start = self.sp.stats()["games_done"]
        while done < num_games:
            self.run_iterations(32)
            ex = self.sp.drain()
            if ex["board"].shape[0]:
                collected.append(ex)
            st = self.sp.stats()
            if st["overflow"]:
                raise _lib.EngineError(f"{st['overflow']} self-play trees overflowed their search path")
            done = st["games_done"] - start
        ex = {k: torch.cat([c[k] for c in collected]) for k in collected[0]} if collected else self.sp.drain()
        if gather:
            ex = gather_examples(ex)
        if with_symmetries:
            ex = expand_symmetries(self.game.engine, ex)
        if not as_tuples:
            return ex
        boards = ex["board"].cpu().numpy()
        pis = ex["pi"].cpu().numpy()
        valids = unpack_mask(ex["valids"]).cpu().numpy()
        win, sd, sur = (ex[k].cpu().numpy() for k in ("winner", "scdiff", "surprise"))
        return [(boards[i], pis[i], win[i], sd[i], valids[i], sur[i]) for i in range(len(boards))]

    def executeEpisode(self):
        return self.executeEpisodes(1)

    def executeIteration(self, num_games, with_symmetries=True, gather=False):
        """Self-play examples of one iteration (Coach.learn's executeEpisode loop,
        Coach.py:123-132) as an ExampleSet, appended to trainExamplesHistory."""
        ex = self.executeEpisodes(num_games, with_symmetries=with_symmetries, as_tuples=False,
                                  gather=gather)
        exset = ExampleSet.from_drain(ex)
        self.trainExamplesHistory.append(exset)
        return exset

    def saveTrainExamples(self, folder=None):
        """Coach.saveTrainExamples (:167-173) without pickle: checkpoint.examples.npz."""
        return self.trainExamplesHistory.save(folder or _arg(self.args, "checkpoint", "checkpoint"))

    def loadTrainExamples(self, folder):
        """Coach.loadTrainExamples (:175-190): read checkpoint.examples.npz."""
        self.trainExamplesHistory = ExampleHistory.load(folder, _arg(self.args, "numItersHistory"),
                                                        device=self.game.engine.device)

    def refresh_network(self):
        """Re-pack the leaf evaluator after the network's weights changed (the fused kernel
        reads a packed copy)."""
        self.sp.evaluator = evaluator_for(self.game.engine, self.nnet, self.B)

    def learn(self, pnet=None, log=None):
        """Coach.learn (Coach.py:102-164): for numIters iterations, numEps self-play games
        (fresh games and trees, as the reference's executeEpisode + reset_all_search_trees),
        the example history saved, the network trained on it, then pitted against the
        previous weights over arenaCompare games (BatchedArena, temp 0, full searches) and
        kept iff it wins >= updateThreshold of the decisive games (under torch.distributed
        every rank's examples are all-gathered first, so all ranks train on the same set);
        checkpoints as
        checkpoint_<i>.pt / best.pt / temp.pt in args.checkpoint. Returns per-iteration
        (nwins, pwins, draws, accepted)."""
        from .NNet import NNetWrapper
        folder = _arg(self.args, "checkpoint", "checkpoint")
        pnet = pnet or NNetWrapper(self.game, dict(self.nnet.args), device=self.nnet.device)
        history = []
        for i in range(1, int(_arg(self.args, "numIters", 1)) + 1):
            if not _arg(self.args, "skipFirstSelfPlay", False) or i > 1:
                self.sp.reset()
                self.executeIteration(int(_arg(self.args, "numEps", self.B)), gather=True)
            self.saveTrainExamples(folder)
            self.nnet.save_checkpoint(folder=folder, filename="temp.pt")
            pnet.load_checkpoint(folder=folder, filename="temp.pt")
            self.nnet.train(self.trainExamplesHistory.merged())
            games = int(_arg(self.args, "arenaCompare", 2))
            arena = BatchedArena(self.game, self.nnet, pnet, self.args, batch=min(games, self.B),
                                 seed=self.seed + i)
            nwins, pwins, draws = arena.playGames(games)
            ok = accept_new_network(nwins, pwins, float(_arg(self.args, "updateThreshold", 0.55)))
            if ok:
                self.nnet.save_checkpoint(folder=folder, filename=f"checkpoint_{i}.pt")
                self.nnet.save_checkpoint(folder=folder, filename="best.pt")
            else:
                self.nnet.load_checkpoint(folder=folder, filename="temp.pt")
            self.refresh_network()
            history.append((nwins, pwins, draws, ok))
            if log:
                log(f"iter {i}: new vs previous {nwins}-{pwins} ({draws} draws) -> "
                    f"{'ACCEPTED' if ok else 'REJECTED'}")
        return history
