"""Training consumer on CPU: GenericNNetWrapper.train's losses and
score-difference targets (:76-80, :171-183) restated independently in numpy, a training run
over a columnar ExampleSet, and the 2-rank gradient all-reduce (gloo) keeping ranks in
lockstep."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from splendor.env import ACTIONS, pack_mask
from splendor.examples import ExampleSet
from splendor.NNet import (NNetWrapper, loss_pi, loss_scdiff_cdf, loss_scdiff_pdf, loss_v,
                           scdiff_targets)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class StubGame:
    """The Game surface NNetWrapper reads (no device engine needed on CPU)."""
    def __init__(self, n=2):
        self.num_players = n

    def getActionSize(self):
        return ACTIONS

    def getBoardSize(self):
        return (32 + 10 * self.num_players + self.num_players ** 2, 7)

    def getMaxScoreDiff(self):
        return 15


def synthetic(E, n=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    R = 32 + 10 * n + n * n
    board = torch.randint(-2, 8, (E, R, 7), generator=g, dtype=torch.int8)
    valid = torch.rand(E, ACTIONS, generator=g) < 0.05
    valid[:, 408] = True
    pi = torch.where(valid, torch.rand(E, ACTIONS, generator=g), torch.zeros(()))
    pi = pi / pi.sum(1, keepdim=True)
    w = (torch.rand(E, generator=g) < 0.5).float() * 2 - 1
    winner = torch.stack([w, -w], 1) if n == 2 else torch.rand(E, n, generator=g)
    scdiff = torch.randint(-20, 21, (E, n), generator=g, dtype=torch.int32)
    surprise = torch.rand(E, n, generator=g)
    return ExampleSet(board, pi, winner, scdiff, pack_mask(valid), surprise)


def test_loss_functions_match_numpy():
    rng = np.random.default_rng(0)
    B, n, D = 5, 2, 31
    t_pi = rng.random((B, ACTIONS)).astype(np.float32)
    o_pi = np.log(rng.random((B, ACTIONS))).astype(np.float32)
    t_v, o_v = rng.random((B, n)).astype(np.float32), rng.random((B, n)).astype(np.float32)
    t_sd = np.zeros((B, D, n), np.float32)
    t_sd[np.arange(B), rng.integers(0, D, B), 0] = 1
    t_sd[np.arange(B), rng.integers(0, D, B), 1] = 1
    o_sd = np.log(rng.dirichlet(np.ones(D), size=(B, n)).transpose(0, 2, 1)).astype(np.float32)
    T = torch.from_numpy
    np.testing.assert_allclose(float(loss_pi(T(t_pi), T(o_pi))), -(t_pi * o_pi).sum() / B, rtol=1e-5)
    np.testing.assert_allclose(float(loss_v(T(t_v), T(o_v))), ((t_v - o_v) ** 2).sum() / (B * n), rtol=1e-5)
    cdf = ((np.cumsum(t_sd, 1) - np.cumsum(np.exp(o_sd), 1)) ** 2).sum() * 0.02 / (B * n)
    np.testing.assert_allclose(float(loss_scdiff_cdf(T(t_sd), T(o_sd))), cdf, rtol=1e-5)
    pdf = -(t_sd * o_sd).sum() * 0.02 / (B * n)
    np.testing.assert_allclose(float(loss_scdiff_pdf(T(t_sd), T(o_sd))), pdf, rtol=1e-5)


def test_scdiff_targets_match_loop():
    sd = torch.tensor([[-20, 3], [15, -15], [0, 16]], dtype=torch.int32)
    got = scdiff_targets(sd, 15).numpy()
    ref = np.zeros((3, 31, 2), np.float32)                 # GenericNNetWrapper.py:76-80
    for i in range(3):
        score_diff = (sd[i].numpy() + 15).clip(0, 30)
        for p in range(2):
            ref[i, score_diff[p], p] = 1
    np.testing.assert_array_equal(got, ref)


def test_train_reduces_loss_on_columnar_examples():
    torch.manual_seed(0)
    ex = synthetic(256)
    w = NNetWrapper(StubGame(), dict(epochs=6, batch_size=32, dropout=0.0, learn_rate=3e-3), device="cpu")

    def full_loss():
        with torch.no_grad():
            w.nnet.eval()
            from splendor.env import unpack_mask
            l = w.losses(ex.board.float(), ex.pi, ex.winner, ex.scdiff, unpack_mask(ex.valids))
            return float(l[0] + 10 * l[1] + l[2] + l[3])

    before = full_loss()
    out = w.train(ex, generator=torch.Generator().manual_seed(1))
    after = full_loss()
    assert set(out) == {"pi", "v", "scdiff"}
    assert after < 0.8 * before, (before, after)
    assert not w.nnet.training


def test_train_accepts_reference_tuples_and_rejects_surprise_weight():
    ex = synthetic(40)
    w = NNetWrapper(StubGame(), dict(epochs=1, batch_size=16), device="cpu")
    assert w.train(ex.to_tuples(), generator=torch.Generator().manual_seed(0)) is not None
    w2 = NNetWrapper(StubGame(), dict(surprise_weight=True), device="cpu")
    with pytest.raises(ValueError):
        w2.train(ex)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, mode="different", bs=16):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "alphazero-general-ori_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from test_train import StubGame, synthetic
    from splendor.NNet import NNetWrapper
    w = NNetWrapper(StubGame(), dict(epochs=1, batch_size=bs, dropout=0.0), device="cpu", seed=0)
    if mode == "different":        # own examples and generator per rank
        gen = torch.Generator().manual_seed(rank)
        w.train(synthetic(64, seed=10 + rank), generator=gen)
        gen_ok = gen.initial_seed() == rank            # the caller's generator is not re-seeded
    else:                          # the same examples and generator on every rank
        gen = torch.Generator().manual_seed(7)
        w.train(synthetic(64, seed=10), generator=gen)
        gen_ok = gen.initial_seed() == 7
    flat = torch.cat([p.detach().reshape(-1) for p in w.nnet.parameters()])
    parts = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(parts, flat)
    info = torch.tensor([int(w.last_shared), int(gen_ok), int(torch.isfinite(flat).all())])
    infos = [torch.zeros_like(info) for _ in range(world)]
    dist.all_gather(infos, info)
    if rank == 0:
        q.put(([p.numpy() for p in parts], [i.tolist() for i in infos]))
    dist.barrier()
    dist.destroy_process_group()


def _two_ranks(mode, bs=16):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode, bs)) for r in range(world)]
    for p in procs:
        p.start()
    parts, infos = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return parts, infos


def test_two_rank_gradient_allreduce_keeps_ranks_identical():
    """Different example sets per rank (own generators): the different-sets path (content
    checksums differ), the ranks stay in lockstep, the callers' generators keep their seeds."""
    parts, infos = _two_ranks("different")
    np.testing.assert_array_equal(parts[0], parts[1])
    assert [i[0] for i in infos] == [0, 0] and [i[1] for i in infos] == [1, 1]
    init = torch.cat([p.detach().reshape(-1) for p in
                      NNetWrapper(StubGame(), {}, device="cpu", seed=0).nnet.parameters()]).numpy()
    assert not np.array_equal(parts[0], init)          # the ranks did train


@pytest.mark.parametrize("bs", (16, 15, 1))
def test_two_rank_shared_set_slices_one_batch(bs):
    """The same example set on both ranks: the shared path (one permutation, rank r trains on
    ids[r::2]); slices of unequal size (15) or empty (batch 1) are weighted by their share,
    so no rank's gradient turns NaN and the ranks stay identical."""
    parts, infos = _two_ranks("shared", bs)
    np.testing.assert_array_equal(parts[0], parts[1])
    assert [i[0] for i in infos] == [1, 1] and all(i[2] == 1 for i in infos)


# ------------------------------------------------------------ parity with the reference
GOLD = os.path.join(ROOT, "tests", "golden")


def _det_weights(sd):
    from test_nnet import deterministic_weights
    return deterministic_weights(sd)


def _reference_training(tag, device):
    """NNetWrapper.train on the examples and injected np.random.choice batches that
    make_golden.py fed GenericNNetWrapper.train (:43-139), starting from the same
    closed-form weights; returns (fixture, per-step losses, final state_dict)."""
    with np.load(os.path.join(GOLD, f"train_{tag}.npz")) as z:
        g = {k: z[k] for k in z.files}
    E, bs, epochs, lr, dropout, vlw, seed = g["args"].tolist()
    n = g["winner"].shape[1]
    w = NNetWrapper(StubGame(n), dict(epochs=int(epochs), batch_size=int(bs), dropout=dropout, learn_rate=lr,
                                      vl_weight=vlw), device=device)
    assert sorted(w.nnet.state_dict()) == list(g["keys"])
    w.nnet.load_state_dict(_det_weights(w.nnet.state_dict()))
    examples = [(g["boards"][i], g["pi"][i], g["winner"][i], g["scdiff"][i], g["valids"][i], g["surprise"][i])
                for i in range(int(E))]
    w._loss_log = []
    torch.manual_seed(int(seed))                  # the generator's dropout masks (CPU)
    w.train(examples, sample_ids=list(g["sample_ids"]))
    sd = {k: v.detach().cpu() for k, v in w.nnet.state_dict().items()}
    return g, np.array(w._loss_log), sd


def _check_training(g, losses, sd, loss_rtol, param_atol, param_rtol):
    assert losses.shape == g["losses"].shape
    np.testing.assert_allclose(losses, g["losses"], rtol=loss_rtol, atol=1e-7)
    worst = 0.0
    for k in g["keys"]:
        ref = g["p:" + k]
        got = sd[k].numpy()
        if not np.issubdtype(ref.dtype, np.floating):
            np.testing.assert_array_equal(got, ref, err_msg=k)
            continue
        err = float(np.abs(got - ref).max()) if ref.size else 0.0
        worst = max(worst, err)
        np.testing.assert_allclose(got, ref, atol=param_atol, rtol=param_rtol, err_msg=k)
    return worst


@pytest.mark.parametrize("tag", ("2p", "2p_dropout", "4p"))
def test_train_matches_reference_wrapper(tag):
    """Six Adam + OneCycleLR steps (2 epochs x 3 batches of 32, lr 1e-3) of NNetWrapper.train
    on CPU against GenericNNetWrapper.train itself (fixture recorded by executing the
    reference, make_golden.py train_fixture): every step's four losses within 1e-6
    relative (measured: <= 2.2e-7) and every parameter / BatchNorm statistic after the last
    step within 1e-5 absolute + 1e-6 relative (measured: <= 3.9e-6 abs, running_var ~60).
    Early Adam steps move a weight by ~lr = 1e-3 each, so a wrong gradient, schedule or
    loss term shows up 100x above the tolerance. 2p_dropout: dropout 0.3, masks drawn
    from the same seeded CPU generator in the reference's order."""
    g, losses, sd = _reference_training(tag, "cpu")
    _check_training(g, losses, sd, loss_rtol=1e-6, param_atol=1e-5, param_rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ("2p", "4p"))
def test_train_matches_reference_wrapper_gpu(tag):
    """The same parity on the GPU (PyTorch-ROCm fp32; dropout off, since device dropout
    masks come from another generator): losses within 1e-5 relative, parameters within
    5e-5 absolute + 1e-5 relative — GEMM reduction orders on the device differ from the
    CPU's (still 20x below one Adam step of lr = 1e-3)."""
    g, losses, sd = _reference_training(tag, "cuda")
    _check_training(g, losses, sd, loss_rtol=1e-5, param_atol=5e-5, param_rtol=1e-5)


def _grad_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "alphazero-general-ori_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splendor.NNet import _allreduce_grads
    ps = [torch.nn.Parameter(torch.zeros(3)) for _ in range(3)]
    ps[0].grad = torch.full((3,), 2.0 + rank)                 # on every rank
    if rank == 0:
        ps[1].grad = torch.full((3,), 4.0)                    # on rank 0 only
    _allreduce_grads(ps)                                      # ps[2]: on no rank
    out = [None if p.grad is None else p.grad.tolist() for p in ps]
    # weighted (uneven per-rank batches): each rank scaled by its share, summed;
    # the flags still travel unscaled, so the no-rank parameter stays None
    qs = [torch.nn.Parameter(torch.zeros(3)) for _ in range(3)]
    qs[0].grad = torch.full((3,), 2.0 + rank)
    if rank == 0:
        qs[1].grad = torch.full((3,), 4.0)
    _allreduce_grads(qs, weight=(0.25, 0.75)[rank])
    out += [None if p.grad is None else p.grad.tolist() for p in qs]
    q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_grads_keeps_absent_gradients_none():
    """a parameter without a gradient on any rank stays grad None (Adam skips it,
    as on one rank); one with a gradient on some rank is averaged with zeros elsewhere."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for out in outs:
        assert out[0] == [2.5] * 3 and out[1] == [2.0] * 3 and out[2] is None
        assert out[3] == [0.25 * 2.0 + 0.75 * 3.0] * 3 and out[4] == [0.25 * 4.0] * 3 and out[5] is None


def test_content_checksum_is_chunk_independent(monkeypatch):
    """The sliced checksum (bounded transient memory) equals the one-slice value."""
    import splendor.NNet as NN
    ex = synthetic(40, seed=3)
    whole = int(NN._content_checksum(ex))
    monkeypatch.setattr(NN, "_CHECKSUM_CHUNK", 997)
    assert int(NN._content_checksum(ex)) == whole
