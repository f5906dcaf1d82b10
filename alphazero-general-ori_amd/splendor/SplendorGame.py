"""The reference's Game plug-in for Splendor (SplendorGame.py:11-86), backed by the HIP engine.

Per-board methods keep the reference's signatures and numpy (R,7) int8 boards, so Arena /
pit / player code written against the reference keeps working (each call is one launch on
a one-board batch). Batched, device-resident work goes through `self.engine`
(splendor.env.SplendorEngine) and splendor.mcts / splendor.selfplay instead.

Chance: getNextState(deterministic=False) / getInitBoard draw their uniforms from Philox
(seed, board 0, stream = call counter) — deterministic for a given seed, where the
reference's Numba RNG is unseeded.
"""
import numpy as np
import torch

from .env import ACTIONS, SplendorEngine, observation_rows, unpack_mask

COLORS = ["white", "blue", "green", "red", "black", "gold"]


class _BoardShim:
    """The slice of the reference's `game.board` jitclass that callers outside the engine
    touch (Arena.py:116,173; SplendorPlayers.py:145-147): token limit + scores of the board
    most recently passed to the game."""

    def __init__(self, game):
        self._g = game
        self.num_players = game.num_players

    def setNumTokenLim(self, n):
        self._g.engine.set_token_limit(n)
        self.NUM_TOKEN_LIMIT = n

    def get_score(self, player):
        return self._g.getScore(self._g._last, player)

    def get_round(self):
        return self._g.getRound(self._g._last)

    def get_state(self):
        return self._g._last

    def copy_state(self, state, copy_or_not=False):
        self._g._last = np.array(state, dtype=np.int8, copy=True) if copy_or_not else state


class SplendorGame:
    def __init__(self, N, is_fill=True, device="cuda", seed=0x5EED):
        self.NUMBER_PLAYERS = N
        self.num_players = N
        self.engine = SplendorEngine(N, device=device)
        self.device = self.engine.device
        self.rows = observation_rows(N)
        self.is_fill = is_fill
        self.seed = seed
        self._calls = 0
        self._last = None
        self.board = _BoardShim(self)

    # ------------------------------------------------------------------ helpers
    def _t(self, board):
        b = np.ascontiguousarray(board, dtype=np.int8).reshape(1, self.rows, 7)
        self._last = b[0]
        return torch.from_numpy(b).to(self.device)

    def _stream(self):
        self._calls += 1
        return self._calls & 0x00FFFFFF

    # ------------------------------------------------------------------ Game API
    def getInitBoard(self):
        st = self.engine.new_state(1)
        self.engine.init(st, seed=self.seed, stream=(6 << 24) | self._stream())
        if not self.is_fill:   # Board(n, is_fill=False): no cards, no nobles (:244-246)
            st[:, 1:25] = 0
            st[:, 31:32 + self.num_players] = 0
        out = st[0].cpu().numpy()
        self._last = out
        return out

    def getBoardSize(self):
        return (self.rows, 7)

    def getActionSize(self):
        return ACTIONS

    def getMaxScoreDiff(self):
        return 15

    def getNextState(self, board, player, action, deterministic=False):
        st = self._t(board)
        nxt = torch.empty(1, dtype=torch.int8, device=self.device)
        self.engine.step(st, torch.tensor([int(action)], dtype=torch.int16, device=self.device),
                         torch.tensor([int(player)], dtype=torch.int8, device=self.device), nxt,
                         deterministic=deterministic, seed=self.seed, stream=(7 << 24) | self._stream())
        out = st[0].cpu().numpy()
        self._last = out
        return out, int(nxt.item())

    def getValidMoves(self, board, player):
        m = self.engine.valid_moves(self._t(board), torch.tensor([int(player)], dtype=torch.int8,
                                                                   device=self.device))
        return unpack_mask(m)[0].cpu().numpy()

    def getGameEnded(self, board, next_player):
        return self.engine.game_ended(self._t(board))[0].cpu().numpy()

    def getScore(self, board, player):
        return int(self.engine.score(self._t(board))[0, player].item())

    def getRound(self, board):
        return int(self.engine.round(self._t(board))[0].item())

    def getCanonicalForm(self, board, player):
        if player == 0:
            return board
        out = self.engine.canonical(self._t(board), torch.tensor([int(player)], dtype=torch.int8,
                                                                  device=self.device))
        return out[0].cpu().numpy()

    def getSymmetries(self, board, pi, valid_actions):
        st = self._t(board)
        pi_t = torch.as_tensor(np.asarray(pi, dtype=np.float32), device=self.device).reshape(1, ACTIONS)
        va = np.zeros(7 * 64, dtype=np.uint8)
        va[:ACTIONS] = np.asarray(valid_actions, dtype=bool)
        words = np.packbits(va.reshape(7, 64)[:, ::-1], axis=1).view(">u8").astype(np.int64).reshape(1, 7)
        s, p, v, present = self.engine.symmetries(st, pi_t, torch.from_numpy(words).to(self.device))
        keep = present[0].cpu().numpy().astype(bool)
        s, p = s[0].cpu().numpy()[keep], p[0].cpu().numpy()[keep]
        v = unpack_mask(v[0]).cpu().numpy()[keep]
        return [(s[i], p[i], v[i]) for i in range(len(s))]

    def stringRepresentation(self, board):
        return np.ascontiguousarray(board, dtype=np.int8).tobytes()

    def getNumberOfPlayers(self):
        return self.NUMBER_PLAYERS

    def moveToString(self, move, current_player=0):
        return move_to_str(int(move))

    def disableReserve(self):
        raise NotImplementedError("ENABLE_ACTION_RESERVE=False is a training-time switch (out of scope)")

    def enableReserve(self):
        pass


def move_to_str(a):
    """Human-readable action name (the action table of SplendorLogic.move_to_str, :59-223)."""
    if a < 12:
        return f"buy tier{a // 4}-card{a % 4}"
    if a < 24:
        return f"reserve tier{(a - 12) // 4}-card{(a - 12) % 4}"
    if a < 27:
        return f"reserve from deck {a - 24}"
    if a < 30:
        return f"buy reserved {a - 27}"
    if a < 60:
        return f"take gems #{a - 30}"
    if a < 290 or 365 <= a < 405:
        return f"exchange gems #{a - 60}"
    if a < 365:
        i = a - 290
        return f"reserve #{i // 5} and give back {COLORS[i % 5]}"
    return "pass" if a == 408 else f"select noble {a - 405}"
