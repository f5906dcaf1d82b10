"""Arena (Arena.py:15-227) on the engine, in two forms.

`Arena(player1, player2, player3, game, args)` keeps the reference's constructor and
playGame / playGames: one game at a time through the Game API with arbitrary player
callables (board -> action), as pit.py and Coach.learn use it.

`BatchedArena(game, nnet1, nnet2, args, batch=B)` is the batched gate: playGames for many
games at once on the device MCTS, as Coach.learn uses it to accept or reject a new network
(Coach.py:150-159).

Reference semantics kept:
* two players, each an MCTS over its own network with a search tree that persists through
  a game and is reset between games (Arena.py:163, MCTS.reset_all_search_trees);
* a move is np.argmax(mcts.getActionProb(canonical, temp=0, force_full_search=True)[0])
  (Coach.py:152-153): the best root visit count, ties broken uniformly
  (MCTS.py:87-92; here the Philox draw (seed, game id, ply), spl_mcts_pick_best);
* game i is played "1 vs 2" (player 1 moves first) when i % 4 in (0, 3), else "2 vs 1"
  (Arena.py:200-203); getNextState with chance (deterministic=False), the result is
  getGameEnded(board)[0], player 0's entry (Arena.py:163-165);
* oneWon / twoWon / draws are counted as at Arena.py:204-214.

Batched form: game slots play in lockstep (every game's mover is ply % n). Each player owns
one BatchedMCTS with one tree per game slot; at each ply only the trees of the games where
that player is to move search (spl_mcts_set_roots_active), the others stay untouched.
Finished games idle (their boards take the no-op pass move, never read again). Chance is
Philox keyed (seed, global game id, ply); deals (seed, game id, 0xFFFFFFFF).
For n > 2 players the reference's player list is [p1, p2] only (Arena.py:86-90, an
IndexError at n = 3 without player3); here seat 0 plays one side and every other seat
the other ([p1] + [p2] * (n-1) and its mirror, the form commented in Arena.py:77-84).
"""
import numpy as np
import torch

from .env import ACTIONS, unpack_mask
from .mcts import BatchedMCTS
from .search import evaluator_for

PASS = 408
DEAL_STREAM = 0xFFFFFFFF


def _arg(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


def one_vs_two(i):
    """Arena.py:200-203: 1 2 2 1  1 2 2 1 ..."""
    return (i % 4 == 0) or (i % 4 == 3)


class BatchedArena:
    def __init__(self, game, nnet1, nnet2, args, batch=None, seed=0x5EED, game_base=0,
                 evaluators=None, check_valid=True):
        self.game, self.args = game, args
        self.e = game.engine
        self.n = self.e.n
        self.B = int(batch or _arg(args, "arenaCompare", 1))
        self.seed, self.game_base = int(seed), int(game_base)
        self.check_valid = check_valid
        if evaluators is None:
            evaluators = (evaluator_for(self.e, nnet1, self.B), evaluator_for(self.e, nnet2, self.B))
        margs = dict(numMCTSSims=int(_arg(args, "numMCTSSims", 100)), cpuct=float(_arg(args, "cpuct", 1.0)),
                     fpu=float(_arg(args, "fpu", 0.0)), prob_fullMCTS=1.0,
                     ratio_fullMCTS=int(_arg(args, "ratio_fullMCTS", 5) or 1),
                     forced_playouts=bool(_arg(args, "forced_playouts", False)), dirichletAlpha=0.0,
                     temperature=list(_arg(args, "temperature", [1.25, 0.8])),
                     tempThreshold=int(_arg(args, "tempThreshold", 10)))
        # the two players' arenas share what is free now (each would otherwise plan 80 % of it)
        budget = None
        if self.e.device.type == "cuda":
            budget = int(0.4 * torch.cuda.mem_get_info(self.e.device)[0])
        self.mcts = [BatchedMCTS(self.e, self.B, margs, evaluators[k], dirichlet_noise=False,
                                 seed=self.mcts_seed(k), board_base=self.game_base, mem_budget=budget)
                     for k in range(2)]
        self.last = None
        self.capacity = {"prunes": 0, "resets": 0, "unexpanded": 0}

    def mcts_seed(self, k):
        return self.seed ^ (k + 1)

    def seats(self, first):
        """seat -> player (0 = player1, 1 = player2) for the games in `first` order."""
        n = self.n
        s = np.where(np.asarray(first)[:, None], np.array([0] + [1] * (n - 1))[None, :],
                     np.array([1] + [0] * (n - 1))[None, :])
        return s

    # ---------------------------------------------------------------- one batch
    def _play_batch(self, g0, G):
        e, B, n, dev = self.e, self.B, self.n, self.e.device
        gid = np.arange(g0, g0 + B)
        alive = torch.from_numpy(np.arange(B) < G).to(dev)
        first = np.array([one_vs_two(int(i)) for i in gid])
        seat_player = torch.from_numpy(self.seats(first)).to(dev)            # [B, n]
        base = self.game_base + g0
        boards = e.new_state(B)
        e.init(boards, None, seed=self.seed, stream=DEAL_STREAM, board_base=base)
        for m in self.mcts:                                                   # fresh trees
            m.set_roots(boards, keep_tree=False, force_full=True)
        done = torch.zeros(B, dtype=torch.bool, device=dev)
        result = torch.zeros((B, n), dtype=torch.float32, device=dev)
        plies = torch.zeros(B, dtype=torch.int32, device=dev)
        action = torch.full((B,), PASS, dtype=torch.int16, device=dev)
        trace = []                                                             # actions per ply
        max_plies = 62 * n * 2 + 8                                             # round cap (:322)
        for ply in range(max_plies):
            cur = ply % n
            player = torch.full((B,), cur, dtype=torch.int8, device=dev)
            canon = e.canonical(boards, player)
            live = alive & ~done
            action.fill_(PASS)
            for k in range(2):
                act = live & (seat_player[:, cur] == k)
                if not bool(act.any()):
                    continue
                a8 = act.to(torch.uint8)
                m = self.mcts[k]
                m.set_roots_active(canon, a8, keep_tree=True, force_full=True)
                m.search()
                m.pick_best(a8, board_base=base, stream=ply, out=action)
            if self.check_valid:                                               # Arena.py:158-159
                valid = unpack_mask(e.valid_moves(canon))
                ok = valid.gather(1, action.long().clamp(0, ACTIONS - 1).unsqueeze(1)).squeeze(1)
                bad = live & ~ok
                if bool(bad.any()):
                    raise AssertionError(f"invalid arena action in games {gid[bad.cpu().numpy()].tolist()}")
            action = torch.where(live, action, torch.full_like(action, PASS))
            trace.append(torch.where(live, action, torch.full_like(action, -1)))
            e.step(boards, action, player=player, deterministic=False, seed=self.seed, stream=ply,
                   board_base=base)
            ended = e.game_ended(boards)
            newly = live & (ended != 0).any(1)
            result[newly] = ended[newly]
            plies[newly] = ply + 1
            done |= newly
            if not bool((alive & ~done).any()):
                break
        acts = torch.stack(trace, 1)[:G].cpu().numpy()
        pad = np.full((G, max_plies - acts.shape[1]), -1, dtype=np.int16)
        return {"game": gid[:G], "one_vs_two": first[:G], "result": result[:G].cpu().numpy(),
                "plies": plies[:G].cpu().numpy(), "score": e.score(boards)[:G].cpu().numpy(),
                "actions": np.concatenate([acts, pad], 1)}

    # ---------------------------------------------------------------- reference API
    def playGames(self, num, verbose=False):
        """Arena.playGames: (oneWon, twoWon, draws) over `num` games; per-game records in
        self.last (game id, one_vs_two, result vector, plies, final scores, actions per ply
        with -1 after the game's end)."""
        recs = []
        for g0 in range(0, num, self.B):
            recs.append(self._play_batch(g0, min(self.B, num - g0)))
        # capacity events of both players' searches (a deviation from the reference's table)
        ev = [m.capacity_events() for m in self.mcts]
        self.capacity = {k: sum(e[k] for e in ev) for k in ev[0]}
        if any(self.capacity.values()):
            import warnings
            warnings.warn(f"BatchedArena capacity events {self.capacity}: some searches ran on pruned trees or "
                          f"left leaves unstored")
        last = {k: np.concatenate([r[k] for r in recs]) for k in recs[0]}
        r0 = last["result"][:, 0]
        ovt = last["one_vs_two"]
        one = int(np.sum(np.where(ovt, r0 == 1.0, r0 == -1.0)))
        two = int(np.sum(np.where(ovt, r0 == -1.0, r0 == 1.0)))
        self.last = last
        return one, two, int(len(r0) - one - two)


class Arena:
    """The reference's sequential Arena (Arena.py:15-227) over the engine-backed Game API:
    player callables take a canonical board and return an action; the tqdm progress bar,
    colours, board records and handicap statistics are console features left out."""

    def __init__(self, player1, player2, player3, game, args=None, display=None, no_record=True):
        self.player1, self.player2, self.player3 = player1, player2, player3
        self.game, self.display = game, display

    def playGame(self, verbose=False, other_way=False, cur_player=None, board=None):
        """Arena.playGame (:66-173): (player 0's result, score of player 0, of player 1)."""
        g = self.game
        if not other_way:
            players = [self.player1, self.player2] if self.player3 is None else \
                [self.player1, self.player2, self.player3]
        else:
            players = [self.player2] + [self.player1] * (g.getNumberOfPlayers() - 1)
        if cur_player is None:
            cur, board = 0, g.getInitBoard()
        else:
            cur = cur_player
        while not g.getGameEnded(board, cur).any():
            canonical = g.getCanonicalForm(board, cur)
            action = players[cur](canonical)
            valids = g.getValidMoves(canonical, 0)
            if valids[action] == 0:                          # Arena.py:158-159
                raise AssertionError(f"player {cur} chose an invalid action {action}")
            board, cur = g.getNextState(board, cur, action)
        from .search import MCTS
        MCTS.reset_all_search_trees()
        return g.getGameEnded(board, cur)[0], g.getScore(board, 0), g.getScore(board, 1)

    def playGames(self, num, verbose=False, cur_player=None, board=None):
        """Arena.playGames (:175-227): player1 moves first in games i % 4 in (0, 3)."""
        one, two, draws = 0, 0, 0
        for i in range(num):
            ovt = one_vs_two(i)
            r, _, _ = self.playGame(verbose=verbose, other_way=not ovt, cur_player=cur_player)
            if r == (1. if ovt else -1.):
                one += 1
            elif r == (-1. if ovt else 1.):
                two += 1
            else:
                draws += 1
        return one, two, draws


def accept_new_network(nwins, pwins, update_threshold):
    """Coach.learn gate (Coach.py:157-164): accept iff pwins + nwins > 0 and
    nwins / (pwins + nwins) >= updateThreshold."""
    return not (pwins + nwins == 0 or float(nwins) / (pwins + nwins) < update_threshold)
