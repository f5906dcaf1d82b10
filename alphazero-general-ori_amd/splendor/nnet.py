"""SplendorNNet under PyTorch-ROCm: the leaf evaluator of the batched search.

The architecture is the reference's SplendorNNet (SplendorNNet.py:56-159: dense layers over
the 7 columns of the (R,7) board with partial max/avg global pooling, policy/value/score-diff
heads). Parameter names follow the reference's state_dict keys so checkpoints saved as plain
state_dicts load with torch.load(weights_only=True).

Inference path (`LeafEvaluator`): eval-mode BatchNorms are folded into per-channel affine
terms once, the score-diff head (training-only) is skipped, and "int8 leaves -> pi, v" runs
as one fused HIP kernel (csrc/nnet.hip, spl_nn_forward; fp32 MFMA) — or, for reference,
as the PyTorch-ROCm FoldedNet, optionally captured in a HIP graph at a fixed batch.
Returns exp(masked log_softmax(pi)) and tanh(v) like GenericNNetWrapper.predict (:141-168).
"""
import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .env import ACTIONS, _ptr


def _lin(i, o):
    m = nn.Linear(i, o)
    nn.init.kaiming_uniform_(m.weight)
    nn.init.zeros_(m.bias)
    return m


class _PoolDense(nn.Module):
    """First `groups*items` features pooled (max, avg) per group; the rest -> Linear(+BN) ->
    ReLU (reference DenseAndPartialGPool, SplendorNNet.py:6-28)."""

    def __init__(self, width, groups, items, bn_channels):
        super().__init__()
        self.groups, self.items = groups, items
        self.dense_part = nn.Sequential(_lin(width - groups * items, width - 2 * groups),
                                        nn.BatchNorm1d(bn_channels))

    def forward(self, x):
        g = self.groups * self.items
        head = x[..., :g].unflatten(-1, (self.groups, self.items))
        return torch.cat([head.amax(-1), head.mean(-1), F.relu(self.dense_part(x[..., g:]))], -1)


def _col_pool(x, length=64, chans=5):
    """Reference FlattenAndPartialGPool(64, 5) (SplendorNNet.py:31-53): over the first 64
    features pool the first 5 channels (max, avg), flatten the rest -> [B, 1, 704]."""
    a, rest = x[..., :length], x[..., length:]
    pooled = a[:, :chans]
    return torch.cat([pooled.amax(1), pooled.mean(1), a[:, chans:].flatten(1), rest.flatten(1)], 1).unsqueeze(1)


class SplendorNNet(nn.Module):
    def __init__(self, n_players=2, action_size=ACTIONS, max_score_diff=15, dropout=0.0):
        super().__init__()
        self.n = n_players
        self.dropout = float(dropout)                       # nn_args['dropout'] (main.py:26)
        self.rows = 32 + 10 * n_players + n_players * n_players
        self.action_size = action_size
        self.scdiff = 2 * max_score_diff + 1
        relu = nn.ReLU
        self.dense2d_1 = nn.Sequential(_lin(self.rows, 128), nn.BatchNorm1d(7), relu(), _lin(128, 128), relu())
        self.partialgpool_1 = _PoolDense(128, 4, 8, 7)
        self.dense2d_3 = nn.Sequential(_lin(128, 128), relu())
        self.dense1d_4 = nn.Sequential(_lin(64 * 4 + 64 * 7, 128), relu())
        self.partialgpool_4 = _PoolDense(128, 4, 4, 1)
        self.dense1d_5 = nn.Sequential(_lin(128, 128), nn.BatchNorm1d(1), relu(), _lin(128, 128), relu())
        self.partialgpool_5 = _PoolDense(128, 4, 4, 1)
        self.output_layers_PI = nn.Sequential(_lin(128, 128), _lin(128, action_size))
        self.output_layers_V = nn.Sequential(_lin(128, 128), _lin(128, n_players))
        self.output_layers_SDIFF = nn.Sequential(_lin(128, 128), _lin(128, n_players * self.scdiff))
        self.register_buffer("lowvalue", torch.FloatTensor([-1e8]))

    def trunk(self, board):
        """SplendorNNet.forward up to the heads (SplendorNNet.py:127-138), dropout where the
        reference applies it (training mode only)."""
        d = lambda t: F.dropout(t, p=self.dropout, training=self.training)  # noqa: E731
        x = board.transpose(-1, -2).reshape(-1, 7, self.rows)
        x = d(self.partialgpool_1(self.dense2d_1(x)))
        x = _col_pool(d(self.dense2d_3(x)))
        x = d(self.partialgpool_4(d(self.dense1d_4(x))))
        return d(self.partialgpool_5(d(self.dense1d_5(x))))

    def forward(self, board, valid):
        """Reference signature: (log_pi, tanh(v), log_softmax(scdiff))."""
        x = self.trunk(board)
        pi = torch.where(valid, self.output_layers_PI(x).squeeze(1), self.lowvalue)
        v = self.output_layers_V(x).squeeze(1)
        sd = self.output_layers_SDIFF(x).squeeze(1).view(-1, self.n, self.scdiff).transpose(1, 2)
        return F.log_softmax(pi, 1), torch.tanh(v), F.log_softmax(sd, 1)


LEGACY_ACTIONS = 406


def remap_policy_head(state_dict):
    """SplendorNNet state_dict with a 406-action policy head -> the 409-action layout.

    The shipped checkpoint predates the select-noble actions (SplendorNNet.py:106-109 sizes
    the head by game.getActionSize(); genbu.pt's head has 406 rows): actions 0-404 are the
    same moves, row 405 was pass. In the 409 layout pass is 408 and rows 405-407
    (select-noble, never legal: DESIGN.md §2) get zero weights. The reference's own
    non-strict loader cannot do this (it copies target -> source for equal shapes and
    truncates otherwise, GenericNNetWrapper.py:215-232). Returns a new dict; 409-row heads
    pass through unchanged."""
    kw, kb = "output_layers_PI.1.weight", "output_layers_PI.1.bias"
    w, b = state_dict[kw], state_dict[kb]
    if w.shape[0] == ACTIONS:
        return dict(state_dict)
    if w.shape[0] != LEGACY_ACTIONS or b.shape[0] != LEGACY_ACTIONS:
        raise ValueError(f"policy head has {w.shape[0]} rows; expected {ACTIONS} or {LEGACY_ACTIONS}")
    nw = w.new_zeros((ACTIONS, w.shape[1]))
    nb = b.new_zeros(ACTIONS)
    nw[:405], nb[:405] = w[:405], b[:405]
    nw[408], nb[408] = w[405], b[405]
    out = dict(state_dict)
    out[kw], out[kb] = nw, nb
    return out


def _bn_affine(bn):
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    return s, bn.bias - bn.running_mean * s


class FoldedNet(nn.Module):
    """Eval-mode inference form of SplendorNNet: BNs folded, no score-diff head."""

    def __init__(self, net):
        super().__init__()
        net = net.eval()
        self.rows = net.rows
        with torch.no_grad():
            l1, bn1, l2 = net.dense2d_1[0], net.dense2d_1[1], net.dense2d_1[3]
            s, t = _bn_affine(bn1)                      # per channel (7)
            self.w1, self.b1 = l1.weight.clone(), l1.bias.clone()
            self.s1, self.t1 = s.view(7, 1).clone(), t.view(7, 1).clone()
            self.w2, self.b2 = l2.weight.clone(), l2.bias.clone()
            pd = net.partialgpool_1.dense_part
            s, t = _bn_affine(pd[1])
            self.wp1, self.bp1 = pd[0].weight.clone(), pd[0].bias.clone()
            self.sp1, self.tp1 = s.view(7, 1).clone(), t.view(7, 1).clone()
            self.w3, self.b3 = net.dense2d_3[0].weight.clone(), net.dense2d_3[0].bias.clone()
            self.w4, self.b4 = net.dense1d_4[0].weight.clone(), net.dense1d_4[0].bias.clone()

            def fold1(lin, bn):                         # BN over 1 channel -> scalar affine
                s, t = _bn_affine(bn)
                return (lin.weight * s).clone(), (lin.bias * s + t).clone()
            self.wp4, self.bp4 = fold1(net.partialgpool_4.dense_part[0], net.partialgpool_4.dense_part[1])
            self.w5a, self.b5a = fold1(net.dense1d_5[0], net.dense1d_5[1])
            self.w5b, self.b5b = net.dense1d_5[3].weight.clone(), net.dense1d_5[3].bias.clone()
            self.wp5, self.bp5 = fold1(net.partialgpool_5.dense_part[0], net.partialgpool_5.dense_part[1])
            h = net.output_layers_PI
            self.wpi1, self.bpi1, self.wpi2, self.bpi2 = (h[0].weight.clone(), h[0].bias.clone(),
                                                          h[1].weight.clone(), h[1].bias.clone())
            h = net.output_layers_V
            self.wv1, self.bv1, self.wv2, self.bv2 = (h[0].weight.clone(), h[0].bias.clone(),
                                                      h[1].weight.clone(), h[1].bias.clone())
        for k, v in list(vars(self).items()):
            if isinstance(v, torch.Tensor):
                delattr(self, k)
                self.register_buffer(k, v.detach().contiguous())

    @staticmethod
    def _pool(x, groups, items, dense):
        g = groups * items
        head = x[..., :g].unflatten(-1, (groups, items))
        return torch.cat([head.amax(-1), head.mean(-1), dense], -1)

    def forward(self, board, valid, transposed=False):
        """board [B,R,7] (or [B,7,R] when transposed=True, as spl_nn_input writes it)."""
        x = board if transposed else board.transpose(-1, -2)              # [B, 7, R]
        x = F.relu(F.linear(x, self.w1, self.b1) * self.s1 + self.t1)
        x = F.relu(F.linear(x, self.w2, self.b2))
        d = F.relu(F.linear(x[..., 32:], self.wp1, self.bp1) * self.sp1 + self.tp1)
        x = self._pool(x, 4, 8, d)
        x = F.relu(F.linear(x, self.w3, self.b3))
        x = _col_pool(x)
        x = F.relu(F.linear(x, self.w4, self.b4))
        x = self._pool(x, 4, 4, F.relu(F.linear(x[..., 16:], self.wp4, self.bp4)))
        x = F.relu(F.linear(x, self.w5a, self.b5a))
        x = F.relu(F.linear(x, self.w5b, self.b5b))
        x = self._pool(x, 4, 4, F.relu(F.linear(x[..., 16:], self.wp5, self.bp5))).squeeze(1)
        pi = F.linear(F.linear(x, self.wpi1, self.bpi1), self.wpi2, self.bpi2)
        pi = torch.softmax(pi.masked_fill(~valid, -1e8), 1)
        v = torch.tanh(F.linear(F.linear(x, self.wv1, self.bv1), self.wv2, self.bv2))
        return pi, v


def _bf16_parts(w):
    """f32 w -> (hi, mid, lo) bf16 bit patterns (int32 holding 16 bits) by truncation, as the
    kernel splits activations; hi + mid + lo == w exactly (lo keeps at most 8 significant bits)."""
    u = w.contiguous().view(torch.int32)
    hi = u & -65536
    r1 = w - hi.view(torch.float32)
    mid = r1.contiguous().view(torch.int32) & -65536
    r2 = (r1 - mid.view(torch.float32)).contiguous().view(torch.int32)
    return [(x >> 16) & 0xFFFF for x in (hi, mid, r2)]


def _split_layer(w, row0=0):
    """The bf16 x 3 copy of a per-column layer: [4][Kp16/16][3][64][8] bf16, element
    (nt, c, p, l, j) = part p of W[32 nt + l % 32 - row0][16 c + 8 (l / 32) + j] (0 outside), as
    float32 storage (two bf16 per float, little-endian). The kernel multiplies these fragments as
    the A operand of v_mfma_f32_32x32x16_bf16 (rows = output channels); row0 = 8 puts
    partialgpool_1's outputs on channels 8..127, behind its 8 pooled channels."""
    N, K = w.shape
    k16 = (K + 15) // 16 * 16
    wp = torch.zeros((128, k16), dtype=torch.float32, device=w.device)
    wp[row0:row0 + N, :K] = w
    parts = torch.stack(_bf16_parts(wp))                           # [3][128][k16]
    # [p][nt][col][c][g][j] -> [nt][c][p][g][col][j]; lane = 32 g + col
    t = parts.view(3, 4, 32, k16 // 16, 2, 8).permute(1, 3, 0, 4, 2, 5).reshape(-1, 2)
    packed = (t[:, 0] | (t[:, 1] << 16)).to(torch.int32)
    return packed.view(torch.float32)


def _split_leaf_layer(w):
    """The bf16 x 3 copy of a per-leaf layer (16x16x32 bf16 MFMA B fragments):
    [NT16][Kp32/32][3][64][8] bf16, element (nt, c, p, l, j) = part p of
    W[16 nt + l % 16][32 c + 8 (l / 16) + j], as float32 storage (two bf16 per float)."""
    N, K = w.shape
    nt = (N + 15) // 16
    k32 = (K + 31) // 32 * 32
    wp = torch.zeros((nt * 16, k32), dtype=torch.float32, device=w.device)
    wp[:N, :K] = w
    parts = torch.stack(_bf16_parts(wp))                           # [3][16 nt][k32]
    # [p][nt][col][c][g][j] -> [nt][c][p][g][col][j]; lane = 16 g + col
    t = parts.view(3, nt, 16, k32 // 32, 4, 8).permute(1, 3, 0, 4, 2, 5).reshape(-1, 2)
    packed = (t[:, 0] | (t[:, 1] << 16)).to(torch.int32)
    return packed.view(torch.float32)


def pack_weights(folded, n_players):
    """Pack a FoldedNet into the layout k_nn_forward reads (include/splendor_amd.h,
    spl_nn_forward): per layer the MFMA B-fragment order — layers 0-3 (32x32x2):
    [NT][S/4][64][4], element (nt, q, l, j) = W[32 nt + (l & 31)][4 q + j + (l >> 5) S],
    S = Kp/2; layers 4-12 (16x16x4, Kp % 16 == 0): [NT][Kp/16][64][4], element (nt, q, l, j)
    = W[16 nt + (l & 15)][16 q + 4 (l >> 4) + j] — then the 0-padded bias; then the
    per-column BN affines; then (16-byte aligned) the bf16 x 3 copies the kernel multiplies:
    layers 0-4 in 32x32x16 fragments (_split_layer; partialgpool_1's rows shifted by 8), layers
    5-12 in 16x16x32 fragments (_split_leaf_layer)."""
    f = folded
    layers = [(f.w1, f.b1), (f.w2, f.b2), (f.wp1, f.bp1), (f.w3, f.b3), (f.w4, f.b4), (f.wp4, f.bp4),
              (f.w5a, f.b5a), (f.w5b, f.b5b), (f.wp5, f.bp5), (f.wpi1, f.bpi1), (f.wpi2, f.bpi2),
              (f.wv1, f.bv1), (f.wv2, f.bv2)]
    parts = []
    with torch.no_grad():
        for li, (w, b) in enumerate(layers):
            N, K = w.shape
            kp = (K + 7) // 8 * 8
            T = 32 if li < 4 else 16
            NT = (N + T - 1) // T
            wp = torch.zeros((NT * T, kp), dtype=torch.float32, device=w.device)
            wp[:N, :K] = w
            if li < 4:      # per-column layers: 32x32x2 fragments, K in 2 halves
                # [nt][col][g][q][j] -> [nt][q][g][col][j]; lane = 32 g + col
                wr = wp.view(NT, T, 2, kp // 8, 4).permute(0, 3, 2, 1, 4)
            else:           # per-leaf layers: 16x16x4 fragments, k groups interleaved by 4
                if kp % 16:
                    raise ValueError(f"per-leaf layer {li}: K={K} is not a multiple of 16")
                # [nt][col][q][g][j] -> [nt][q][g][col][j]; lane = 16 g + col
                wr = wp.view(NT, T, kp // 16, 4, 4).permute(0, 2, 3, 1, 4)
            parts.append(wr.reshape(-1))
            bp = torch.zeros(NT * T, dtype=torch.float32, device=w.device)
            bp[:N] = b
            parts.append(bp)
        parts += [f.s1.reshape(7), f.t1.reshape(7), f.sp1.reshape(7), f.tp1.reshape(7)]
        pad = -sum(p.numel() for p in parts) % 4                    # 16-byte aligned split copies
        parts.append(torch.zeros(pad, dtype=torch.float32, device=f.w1.device))
        parts += [_split_layer(w, row0=8 if li == 2 else 0) for li, (w, _) in enumerate(layers[:5])]
        parts += [_split_leaf_layer(w) for w, _ in layers[5:]]
        out = torch.cat([p.float() for p in parts]).contiguous()
    want = _lib.lib().spl_nn_packed_floats(n_players)
    if out.numel() != want:
        raise _lib.EngineError(f"packed network has {out.numel()} floats, engine expects {want}")
    return out


class FusedNet:
    """SplendorNNet inference through the fused HIP kernel (spl_nn_forward): int8 leaf
    boards + packed masks -> (softmax policy, tanh value), all fp32."""

    def __init__(self, net, n_players, device):
        self.n = n_players
        self.device = torch.device(device)
        self.w = pack_weights(FoldedNet(net).to(self.device).eval(), n_players)

    def __call__(self, leaf_state, leaf_mask, pi=None, v=None, index=None, count=None):
        """index / count (device int32, spl_mcts_select_compact's segmented list: B entries and
        ceil(B / 64) segment counts): evaluate only the listed rows (other rows of pi / v are
        left as they are)."""
        B = leaf_state.shape[0]
        pi = pi if pi is not None else torch.empty((B, ACTIONS), dtype=torch.float32, device=self.device)
        v = v if v is not None else torch.empty((B, self.n), dtype=torch.float32, device=self.device)
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        if index is None:
            _lib.check(_lib.lib().spl_nn_forward(self.n, B, _ptr(leaf_state), _ptr(leaf_mask), _ptr(self.w),
                                                 _ptr(pi), _ptr(v), s), "spl_nn_forward")
        else:
            _lib.check(_lib.lib().spl_nn_forward_indexed(self.n, B, _ptr(leaf_state), _ptr(leaf_mask), _ptr(index),
                                                         _ptr(count), _ptr(self.w), _ptr(pi), _ptr(v), s),
                       "spl_nn_forward_indexed")
        return pi, v


def random_net(n_players=2, seed=0, device="cuda"):
    """Seeded random-init SplendorNNet (no pretrained weights load safely)."""
    g = torch.random.fork_rng(devices=[])
    with g:
        torch.manual_seed(seed)
        net = SplendorNNet(n_players)
    return net.to(device).eval()


class LeafEvaluator:
    """Batched nnet.predict for the search (GenericNNetWrapper.predict, :141-168): int8 leaf
    boards + packed masks -> (pi f32 [B,409], v f32 [B,n]).

    fused=True (default): one spl_nn_forward launch (the fused HIP network kernel).
    fused=False: the PyTorch-ROCm FoldedNet (hipBLASLt GEMMs; reference for the tests),
    optionally captured in a HIP graph."""

    def __init__(self, engine, net, B, use_graph=True, fused=True):
        self.e = engine
        self.B = B
        self.fused = FusedNet(net, engine.n, engine.device) if fused else None
        self.net = FoldedNet(net).to(engine.device).eval()
        dev = engine.device
        if fused:
            self.pi_buf = torch.empty((B, ACTIONS), dtype=torch.float32, device=dev)
            self.v_buf = torch.empty((B, engine.n), dtype=torch.float32, device=dev)
        self.x = torch.zeros((B, 7, engine.rows), dtype=torch.float32, device=dev)   # transposed
        self.valid = torch.zeros((B, ACTIONS), dtype=torch.bool, device=dev)
        self.use_graph = use_graph
        self.graph = None
        self.pi = self.v = None
        self._state_ptr = self._mask_ptr = None

    def _convert(self, leaf_state, leaf_mask):
        _lib.check(self.e.L.spl_nn_input(self.e.ctx, self.B, _ptr(leaf_state), _ptr(leaf_mask),
                                         _ptr(self.x), C.c_void_p(self.valid.data_ptr()), self.e._s()),
                   "spl_nn_input")

    @torch.no_grad()
    def _run(self, leaf_state, leaf_mask):
        self._convert(leaf_state, leaf_mask)
        return self.net(self.x, self.valid, transposed=True)

    @property
    def indexed(self):
        """The fused kernel can evaluate a compacted leaf list (spl_nn_forward_indexed)."""
        return self.fused is not None

    @torch.no_grad()
    def __call__(self, leaf_state, leaf_mask, leaf_valid=None, index=None, count=None):
        if self.fused is not None:
            return self.fused(leaf_state, leaf_mask, self.pi_buf, self.v_buf, index=index, count=count)
        if not self.use_graph:
            return self._run(leaf_state, leaf_mask)
        key = (leaf_state.data_ptr(), leaf_mask.data_ptr())
        if self.graph is None or key != (self._state_ptr, self._mask_ptr):
            s = torch.cuda.Stream(self.e.device)
            s.wait_stream(torch.cuda.current_stream(self.e.device))
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._run(leaf_state, leaf_mask)
            torch.cuda.current_stream(self.e.device).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.pi, self.v = self._run(leaf_state, leaf_mask)
            self._state_ptr, self._mask_ptr = key
        self.graph.replay()
        return self.pi, self.v
