"""NeuralNet plug-in for Splendor (NNet.py:1-9 + GenericNNetWrapper: predict, train,
checkpoints).

`predict` is the reference's batch-1 call; self-play and arenas evaluate leaves in batches
through splendor.nnet.LeafEvaluator instead (fused HIP kernel). `train` is
GenericNNetWrapper.train (:43-139) fed straight from columnar device examples
(splendor.examples.ExampleSet: no per-sample unpickling, targets built on device), with the
same losses (:171-183), Adam + OneCycleLR schedule and batch sampling; under
torch.distributed the gradients are averaged across ranks in one flat bucket (RCCL
all-reduce) so every rank keeps identical weights. Checkpoints are read with
torch.load(weights_only=True); files that pickle whole model objects (like the reference's
genbu.pt) are refused by that loader and are reported, never unpickled.
"""
import os

import numpy as np
import torch
import torch.optim as optim

from .env import unpack_mask
from .examples import ExampleSet
from .nnet import SplendorNNet, remap_policy_head

DEFAULT_NN_ARGS = dict(learn_rate=0.0003, dropout=0.3, epochs=2, batch_size=32, vl_weight=10.0,
                       surprise_weight=False)          # main.py:24-33, 121-127


# ---------------------------------------------------------------- losses (:171-183)
def loss_pi(targets, outputs):
    return -torch.sum(targets * outputs) / targets.size()[0]


def loss_v(targets, outputs):
    return torch.sum((targets - outputs) ** 2) / (targets.size()[0] * targets.size()[-1])


def loss_scdiff_cdf(targets, outputs):
    l2_diff = torch.square(torch.cumsum(targets, axis=1) - torch.cumsum(torch.exp(outputs), axis=1))
    return 0.02 * torch.sum(l2_diff) / (targets.size()[0] * targets.size()[-1])


def loss_scdiff_pdf(targets, outputs):
    cross_entropy = -torch.sum(torch.mul(targets, outputs))
    return 0.02 * cross_entropy / (targets.size()[0] * targets.size()[-1])


def scdiff_targets(scdiff, max_diff):
    """One-hot score-difference targets [B, 2*max_diff+1, n] (:76-80), built on device."""
    B, n = scdiff.shape
    idx = (scdiff.long() + max_diff).clamp(0, 2 * max_diff)
    t = torch.zeros((B, 2 * max_diff + 1, n), dtype=torch.float32, device=scdiff.device)
    t.scatter_(1, idx.unsqueeze(1), 1.0)
    return t


def _dist_world():
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return None, 0, 1
    return dist, dist.get_rank(), dist.get_world_size()


def _agreed_batch_count(batch_count, device):
    """Every rank must make the same number of gradient all-reduces: the minimum over ranks
    of E // batch_size (ranks may hold different example counts)."""
    dist, _, world = _dist_world()
    if world == 1:
        return batch_count
    t = torch.tensor([batch_count], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def _batch_generator(device):
    """Batch sampling stream, seeded from the global torch RNG (itself unseeded unless the
    caller seeds it, like the reference's np.random.choice). Under torch.distributed rank
    0's seed is broadcast, so every rank draws the same permutations (see `train`)."""
    dist, _, world = _dist_world()
    seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
    if world > 1:
        seed = seed.to(device)
        dist.broadcast(seed, src=0)
    g = torch.Generator(device=device)
    g.manual_seed(int(seed.item()))
    return g


_CHECKSUM_CHUNK = 1 << 24     # bytes hashed per slice: transient memory independent of the set size


def _content_checksum(ex):
    """64-bit checksum of an ExampleSet's contents (every column's bytes, position-weighted;
    integer sums wrap identically on any device), so ranks can tell whether they hold the
    same examples — equal counts alone do not say that. Hashed in slices of _CHECKSUM_CHUNK
    bytes with a running accumulator (the position weights continue across slices), so the
    int64 temporaries stay ~400 MB at most however many examples the set holds."""
    h = torch.zeros((), dtype=torch.int64, device=ex.board.device)
    for k, col in enumerate((ex.board, ex.pi, ex.winner, ex.scdiff, ex.valids, ex.surprise)):
        b = col.contiguous().reshape(-1).view(torch.uint8)
        s = torch.zeros((), dtype=torch.int64, device=b.device)
        for off in range(0, b.numel(), _CHECKSUM_CHUNK):
            part = b[off:off + _CHECKSUM_CHUNK].to(torch.int64)
            w = torch.arange(off + 1, off + part.numel() + 1, dtype=torch.int64, device=b.device) * 0x9E3779B1 \
                + (k + 1) * 0x7F4A7C15
            s += (part * w).sum()
        h = h * 0x100000001B3 + s
    return h


def _same_everywhere(ex, device):
    """True when every rank holds the same examples (Coach.learn all-gathers, so ranks hold
    the same set): the example count and a content checksum agree across ranks."""
    dist, _, world = _dist_world()
    if world == 1:
        return True
    h = _content_checksum(ex).to(device)
    t = torch.stack([torch.tensor(len(ex), dtype=torch.int64, device=device), h])
    t = torch.cat([t, -t])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t[0]) == -int(t[2]) == len(ex) and int(t[1]) == -int(t[3]) == int(h)


def _allreduce_grads(params, weight=None):
    """Sum (weight given: each rank's gradients scaled by its share of the global batch) or
    average (weight None) the gradients over ranks in one flat bucket (the model is ~1.25 MB
    of fp32). A parameter without a gradient on this rank contributes zeros to the bucket;
    one that got no gradient on ANY rank (a per-parameter presence flag travels in the same
    all-reduce) is left with grad None afterwards, so Adam skips it exactly as a single-rank
    run does."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return
    had = [p.grad is not None for p in params]
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    grads = [p.grad for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads])
    if weight is not None:
        flat *= weight
    presence = torch.tensor(had, dtype=flat.dtype, device=flat.device)
    flat = torch.cat([flat, presence])
    dist.all_reduce(flat)
    present = (flat[-len(params):] > 0).tolist() if params else []
    flat = flat[:-len(params)] if params else flat
    if weight is None:
        flat /= dist.get_world_size()
    off = 0
    for p, g, keep in zip(params, grads, present):
        if keep:
            g.copy_(flat[off:off + g.numel()].view_as(g))
        else:
            p.grad = None
        off += g.numel()


class NNetWrapper:
    def __init__(self, game, nn_args=None, use_exchange=True, device=None, seed=0):
        self.args = dict(DEFAULT_NN_ARGS, **(nn_args or {}))
        self.device = torch.device(device) if device else game.engine.device
        torch.manual_seed(seed)
        self.nnet = SplendorNNet(game.num_players, dropout=self.args["dropout"]).to(self.device).eval()
        self.action_size = game.getActionSize()
        self.rows = game.getBoardSize()[0]
        self.max_diff = game.getMaxScoreDiff()
        self.num_players = game.num_players
        self.optimizer = None

    @torch.no_grad()
    def predict(self, board, valid_actions):
        """GenericNNetWrapper.predict (:141-168): (exp(log_pi)[409], tanh(v)[n]) as numpy."""
        self.nnet.eval()
        b = torch.as_tensor(np.asarray(board, dtype=np.float32), device=self.device).reshape(1, self.rows, 7)
        va = torch.as_tensor(np.asarray(valid_actions, dtype=bool), device=self.device).reshape(1, -1)
        log_pi, v, _ = self.nnet(b, va)
        return torch.exp(log_pi)[0].cpu().numpy(), v[0].cpu().numpy()

    # ------------------------------------------------------------ training (:43-139)
    def losses(self, boards, pis, vs, scdiffs, valids):
        """(l_pi, l_v, l_scdiff_cdf, l_scdiff_pdf) of one batch of device tensors."""
        out_pi, out_v, out_sd = self.nnet(boards, valids)
        t_sd = scdiff_targets(scdiffs, self.max_diff)
        return (loss_pi(pis, out_pi), loss_v(vs, out_v), loss_scdiff_cdf(t_sd, out_sd),
                loss_scdiff_pdf(t_sd, out_sd))

    def train(self, examples, generator=None, sample_ids=None, shared=None):
        """One GenericNNetWrapper.train call over `examples` (ExampleSet, or the reference's
        list of tuples): epochs x (len // batch_size) Adam steps on batches sampled without
        replacement, total loss l_pi + vl_weight * l_v + l_cdf + l_pdf, OneCycleLR stepped
        per batch. Returns the mean of each loss over the last epoch.

        sample_ids: the batches themselves (one index array of batch_size per step, epochs x
        batch_count of them) — the reference's np.random.choice draws (:70) injected, as the
        parity tests do; then nothing is drawn from any RNG here, so dropout masks come from
        the global torch generator in the reference's order.

        Across ranks (torch.distributed): with the same example set on every rank (what
        Coach.learn's all-gather leaves) all ranks draw the same permutation per step and
        rank r trains on its slice ids[r::world] of the batch; each rank's gradients are
        scaled by its slice's share of the batch and summed in one all-reduce, i.e. the
        gradient of the mean loss over the whole batch (slices may differ in size, an empty
        one contributes zeros): the step count and the samples per step are the
        reference's (a global batch of batch_size; BatchNorm statistics are per rank).
        Ranks holding different sets sample their own batches of batch_size from a per-call
        generator seeded by a draw from `generator` mixed with the rank (the caller's
        generator only advances by that draw), gradients averaged; the step count is the
        minimum over ranks, so no rank waits in an all-reduce the others never enter.
        shared: None detects it (example count and content checksum agree on every rank);
        True / False force a path (every rank must pass the same)."""
        if not isinstance(examples, ExampleSet):
            examples = ExampleSet.from_tuples(list(examples))
        if self.args["surprise_weight"]:
            # the reference's weights are [E, n] (one per player) and np.random.choice
            # rejects a 2-D p, so surprise weighting cannot run there either
            raise ValueError("surprise_weight: per-example surprise is a vector (reference raises)")
        ex = examples.to(self.device)
        E, bs, epochs = len(ex), int(self.args["batch_size"]), int(self.args["epochs"])
        dist, rank, world = _dist_world()
        if shared is None:
            shared = _same_everywhere(ex, self.device)
        self.last_shared = bool(shared)
        batch_count = _agreed_batch_count(E // bs, self.device)
        if batch_count == 0:
            return None
        if sample_ids is not None:
            sample_ids = [torch.as_tensor(np.asarray(i, dtype=np.int64), device=self.device) for i in sample_ids]
            if len(sample_ids) != epochs * batch_count or any(len(i) != bs for i in sample_ids):
                raise ValueError(f"sample_ids: need {epochs * batch_count} batches of {bs}")
        params = list(self.nnet.parameters())
        if self.optimizer is None:
            self.optimizer = optim.Adam(params, lr=self.args["learn_rate"])
        scheduler = optim.lr_scheduler.OneCycleLR(self.optimizer, max_lr=self.args["learn_rate"],
                                                  steps_per_epoch=batch_count, epochs=epochs)
        gen = None if sample_ids is not None else (generator or _batch_generator(self.device))
        if gen is not None and not shared and world > 1:    # different sets: decorrelate the ranks
            s0 = int(torch.randint(0, 2 ** 62, (1,), generator=gen, device=gen.device).item())
            gen = torch.Generator(device=self.device)
            gen.manual_seed((s0 ^ (0x9E3779B97F4A7C15 * (rank + 1))) & (2 ** 63 - 1))
        means, step = None, 0
        for _ in range(epochs):
            self.nnet.train()
            acc = torch.zeros(3, dtype=torch.float64, device=self.device)
            for _ in range(batch_count):
                if sample_ids is not None:
                    ids = sample_ids[step]
                else:
                    ids = torch.randperm(E, generator=gen, device=self.device)[:bs]
                weight = None
                if shared and world > 1:
                    ids = ids[rank::world]
                    weight = len(ids) / bs       # this slice's share of the global batch
                step += 1
                self.optimizer.zero_grad(set_to_none=True)
                if len(ids) == 0:                # (batch_size < world: nothing on this rank)
                    _allreduce_grads(params, weight)
                    self.optimizer.step()
                    scheduler.step()
                    continue
                boards = ex.board.index_select(0, ids).float()
                valids = unpack_mask(ex.valids.index_select(0, ids))
                pis = ex.pi.index_select(0, ids)
                vs = ex.winner.index_select(0, ids)
                sds = ex.scdiff.index_select(0, ids)
                l_pi, l_v, l_c, l_p = self.losses(boards, pis, vs, sds, valids)
                total = l_pi + self.args["vl_weight"] * l_v + l_c + l_p
                total.backward()
                _allreduce_grads(params, weight)
                self.optimizer.step()
                scheduler.step()
                acc += torch.stack([l_pi.detach(), l_v.detach(), (l_c + l_p).detach()]).double()
                if self._loss_log is not None:
                    self._loss_log.append([float(x.detach()) for x in (l_pi, l_v, l_c, l_p)])
            means = (acc / batch_count).tolist()
        self.nnet.eval()
        return {"pi": means[0], "v": means[1], "scdiff": means[2]}

    last_shared = None   # the path the last train() call took across ranks
    _loss_log = None     # list: per-step (l_pi, l_v, l_cdf, l_pdf) appended by train (tests)

    # ------------------------------------------------------------ checkpoints
    def save_checkpoint(self, folder="checkpoint", filename="checkpoint.pt", additional_keys=None):
        os.makedirs(folder, exist_ok=True)
        data = {"state_dict": self.nnet.state_dict()}
        data.update(additional_keys or {})
        torch.save(data, os.path.join(folder, filename))

    def load_checkpoint(self, folder="checkpoint", filename="checkpoint.pt"):
        path = os.path.join(folder, filename)
        try:
            data = torch.load(path, map_location=self.device, weights_only=True)
        except Exception as e:  # refused by the safe loader: never fall back to unpickling
            raise RuntimeError(f"{path}: not loadable with torch.load(weights_only=True) ({type(e).__name__})") from e
        sd = data["state_dict"] if isinstance(data, dict) and "state_dict" in data else data
        self.nnet.load_state_dict(remap_policy_head(sd))   # 406-action checkpoints -> 409
        self.nnet.eval()
        return data
