"""Batched, device-resident Splendor environment over libsplendor_amd.so.

Each method is one stream-ordered HIP launch over B boards held in HBM as torch tensors
(torch is only the allocator / stream provider here; all compute is the HIP engine).
Shapes follow the reference's per-board API, batched on a leading dimension:
    state  int8  [B, R, 7]   (SplendorLogicNumba.Board.state, :291-303)
    player int8  [B]
    mask   int64 [B, 7]      (409 legality bits, packed; unpack with `unpack_mask`)
"""
import ctypes as C

import torch

from . import _lib

ACTIONS = 409
MASK_WORDS = 7


def observation_rows(n_players):
    return 32 + 10 * n_players + n_players * n_players


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_BIT = None


def pack_mask(valid):
    """bool [...,409] -> [...,7] int64 packed words (bit i of word k = action 64k+i), the
    engine's mask layout; inverse of unpack_mask."""
    global _BIT
    if _BIT is None or _BIT.device != valid.device:
        _BIT = torch.arange(64, device=valid.device, dtype=torch.int64)
    pad = torch.zeros((*valid.shape[:-1], MASK_WORDS * 64), dtype=torch.int64, device=valid.device)
    pad[..., :ACTIONS] = valid.to(torch.int64)
    return (pad.view(*valid.shape[:-1], MASK_WORDS, 64) << _BIT).sum(-1)


def unpack_mask(mask):
    """[...,7] packed words -> bool [...,409] (on the same device)."""
    global _BIT
    if _BIT is None or _BIT.device != mask.device:
        _BIT = torch.arange(64, device=mask.device, dtype=torch.int64)
    bits = (mask.to(torch.int64).unsqueeze(-1) >> _BIT) & 1
    return bits.reshape(*mask.shape[:-1], MASK_WORDS * 64)[..., :ACTIONS].bool()


class SplendorEngine:
    """A rules context (players, token limit) bound to one device."""

    def __init__(self, n_players=2, token_limit=10, device="cuda"):
        self.L = _lib.lib()
        self.n = int(n_players)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.NativeEngineMissing("the Splendor engine runs on a HIP device only")
        h = C.c_void_p()
        _lib.check(self.L.spl_ctx_create(self.n, int(token_limit), C.byref(h)), "spl_ctx_create")
        self.ctx = h
        self.rows = observation_rows(self.n)
        self.S = 7 * self.rows

    def __del__(self):
        if getattr(self, "ctx", None) is not None:
            self.L.spl_ctx_destroy(self.ctx)
            self.ctx = None

    # ------------------------------------------------------------- allocation helpers
    def new_state(self, B):
        return torch.zeros((B, self.rows, 7), dtype=torch.int8, device=self.device)

    def _s(self):
        return _stream(self.device)

    @staticmethod
    def _chance(uniforms):
        if uniforms is None:
            return None, 0
        assert uniforms.dtype == torch.float64 and uniforms.dim() == 2 and uniforms.is_contiguous()
        return _ptr(uniforms), uniforms.shape[1]

    # ------------------------------------------------------------- Game API, batched
    def init(self, state, player=None, seed=0, stream=0xFFFFFFFF, board_base=0, uniforms=None):
        """Board.init_game on every board (getInitBoard)."""
        up, us = self._chance(uniforms)
        _lib.check(self.L.spl_init(self.ctx, state.shape[0], _ptr(state), _ptr(player), up, us,
                                   seed, stream, board_base, self._s()), "spl_init")
        return state

    def valid_moves(self, state, player=None, out=None):
        B = state.shape[0]
        out = out if out is not None else torch.empty((B, MASK_WORDS), dtype=torch.int64, device=self.device)
        _lib.check(self.L.spl_valid_moves(self.ctx, B, _ptr(state), _ptr(player), _ptr(out), self._s()),
                   "spl_valid_moves")
        return out

    def step(self, state, action, player=None, next_player=None, deterministic=False, seed=0,
             stream=0, board_base=0, uniforms=None, err=None):
        """make_move in place (getNextState). action: int16 [B]."""
        B = state.shape[0]
        up, us = self._chance(uniforms)
        _lib.check(self.L.spl_step(self.ctx, B, _ptr(state), _ptr(player), _ptr(action),
                                   _ptr(next_player), int(bool(deterministic)), up, us, seed, stream,
                                   board_base, _ptr(err), self._s()), "spl_step")
        return next_player

    def game_ended(self, state, out=None):
        B = state.shape[0]
        out = out if out is not None else torch.empty((B, self.n), dtype=torch.float32, device=self.device)
        _lib.check(self.L.spl_game_ended(self.ctx, B, _ptr(state), _ptr(out), self._s()), "spl_game_ended")
        return out

    def canonical(self, state, player, out=None):
        out = out if out is not None else torch.empty_like(state)
        _lib.check(self.L.spl_canonical(self.ctx, state.shape[0], _ptr(state), _ptr(player), _ptr(out),
                                        self._s()), "spl_canonical")
        return out

    def score(self, state):
        out = torch.empty((state.shape[0], self.n), dtype=torch.int32, device=self.device)
        _lib.check(self.L.spl_score(self.ctx, state.shape[0], _ptr(state), _ptr(out), self._s()), "spl_score")
        return out

    def round(self, state):
        out = torch.empty((state.shape[0],), dtype=torch.int32, device=self.device)
        _lib.check(self.L.spl_round(self.ctx, state.shape[0], _ptr(state), _ptr(out), self._s()), "spl_round")
        return out

    def tree_step(self, parent, action, child=None, err=None):
        child = child if child is not None else torch.empty_like(parent)
        _lib.check(self.L.spl_tree_step(self.ctx, parent.shape[0], _ptr(parent), _ptr(action), _ptr(child),
                                        _ptr(err), self._s()), "spl_tree_step")
        return child

    def set_token_limit(self, n):
        """Board.setNumTokenLim (SplendorLogicNumba.py:214-215)."""
        _lib.check(self.L.spl_ctx_set_token_limit(self.ctx, int(n)), "spl_ctx_set_token_limit")

    def symmetries(self, state, pi, valid):
        """Board.get_symmetries for E examples -> (state [E,K,R,7], pi [E,K,409],
        valid [E,K,7], present [E,K]) with K = 10 + 2n (reference order)."""
        E, K = state.shape[0], 10 + 2 * self.n
        dev = self.device
        os_ = torch.empty((E, K, self.rows, 7), dtype=torch.int8, device=dev)
        op = torch.empty((E, K, ACTIONS), dtype=torch.float32, device=dev)
        ov = torch.empty((E, K, MASK_WORDS), dtype=torch.int64, device=dev)
        pr = torch.empty((E, K), dtype=torch.uint8, device=dev)
        _lib.check(self.L.spl_symmetries(self.ctx, E, _ptr(state), _ptr(pi.contiguous()), _ptr(valid.contiguous()),
                                         _ptr(os_), _ptr(op), _ptr(ov), _ptr(pr), self._s()), "spl_symmetries")
        return os_, op, ov, pr

    def rollout_step(self, state, player, mask_out, action_out, ended_out, games_done, seed, step,
                     board_base=0):
        _lib.check(self.L.spl_rollout_step(self.ctx, state.shape[0], _ptr(state), _ptr(player),
                                           _ptr(mask_out), _ptr(action_out), _ptr(ended_out),
                                           _ptr(games_done), seed, step, board_base, self._s()),
                   "spl_rollout_step")

    def rollout_run(self, K, state, player, mask_out, action_out, ended_out, games_done, seed, step0,
                    board_base=0):
        """K fused moves in one launch; outputs stacked by move ([K][B]...)."""
        _lib.check(self.L.spl_rollout_run(self.ctx, state.shape[0], int(K), _ptr(state), _ptr(player),
                                          _ptr(mask_out), _ptr(action_out), _ptr(ended_out),
                                          _ptr(games_done), seed, step0, board_base, self._s()),
                   "spl_rollout_run")


class RolloutBatch:
    """B boards of random-policy self-play, stepped by one fused launch per step
    (BASELINE config 2). All buffers live in HBM for the whole run."""

    def __init__(self, engine, B, seed=0x5EED, board_base=0):
        self.e = engine
        self.B = B
        self.seed = seed
        self.board_base = board_base
        dev = engine.device
        self.state = engine.new_state(B)
        self.player = torch.zeros(B, dtype=torch.int8, device=dev)
        self.mask = torch.zeros((B, MASK_WORDS), dtype=torch.int64, device=dev)
        self.action = torch.zeros(B, dtype=torch.int16, device=dev)
        self.ended = torch.zeros((B, engine.n), dtype=torch.float32, device=dev)
        self.games = torch.zeros(B, dtype=torch.int32, device=dev)
        self.t = 0
        engine.init(self.state, self.player, seed=seed, stream=0xFFFFFFFF, board_base=board_base)

    def step(self):
        self.e.rollout_step(self.state, self.player, self.mask, self.action, self.ended, self.games,
                            self.seed, self.t, self.board_base)
        self.t += 1

    def launcher(self, K, out):
        """A prebuilt launch of `run(K, out=out)`: every argument but the step counter is
        converted once, so a timed region pays one ctypes call per launch (bench.py)."""
        e = self.e
        fn = e.L.spl_rollout_run
        head = (e.ctx, self.B, int(K), _ptr(self.state), _ptr(self.player), _ptr(out["mask"]),
                _ptr(out["action"]), _ptr(out["ended"]), _ptr(self.games), self.seed)
        tail = (self.board_base, e._s())

        def launch():
            rc = fn(*head, self.t, *tail)
            if rc:
                _lib.check(rc, "spl_rollout_run")
            self.t += K
        return launch

    def run(self, K, masks=True, out=None):
        """K moves in one launch (boards stay on chip); returns the stacked per-move outputs
        {"mask": [K,B,7] or None, "action": [K,B], "ended": [K,B,n]} (reused if `out`)."""
        B, dev, n = self.B, self.e.device, self.e.n
        if out is None or out["action"].shape[0] != K:
            out = {"mask": torch.empty((K, B, MASK_WORDS), dtype=torch.int64, device=dev) if masks else None,
                   "action": torch.empty((K, B), dtype=torch.int16, device=dev),
                   "ended": torch.empty((K, B, n), dtype=torch.float32, device=dev)}
        self.e.rollout_run(K, self.state, self.player, out["mask"], out["action"], out["ended"], self.games,
                           self.seed, self.t, self.board_base)
        self.t += K
        return out
