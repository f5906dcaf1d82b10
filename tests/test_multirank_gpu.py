"""The product's multi-rank self-play path on one GPU: two processes on cuda:0
over a gloo group, each running a SelfPlay shard (board_base = rank x B) with SplendorNNet
leaves from the fused kernel, `broadcast_network` (rank 1 starts from other weights and
must search with rank 0's) and `gather_examples` (one packed-record all-gather) on the
examples its games really produced. The gathered set, ordered by (board id, game, index),
must equal bit for bit the examples of ONE process running all 2B games — the claim that
results do not depend on the GPU count (the reference plays the same games sequentially,
Coach.py:117-124). RCCL itself is only exercised by the multi-GPU bench on an 8-GPU node.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, SIMS, ITERS = 48, 16, 3000
ARGS = dict(numMCTSSims=SIMS, cpuct=2.5, fpu=0.3, prob_fullMCTS=0.5, ratio_fullMCTS=4, forced_playouts=False,
            dirichletAlpha=0.3, temperature=[1.25, 0.8], tempThreshold=10)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _play(rank, games, net_seed, dist_on):
    from splendor.env import SplendorEngine
    from splendor.nnet import LeafEvaluator, random_net
    from splendor.selfplay import SelfPlay, broadcast_network, gather_examples
    dev = torch.device("cuda", 0)
    eng = SplendorEngine(2, device=dev)
    net = random_net(2, seed=net_seed, device=dev)
    if dist_on:
        broadcast_network(net)
    ev = LeafEvaluator(eng, net, games, use_graph=False)
    # an explicit arena budget: the default (80 % of the free HBM, read at construction)
    # races when two processes share the GPU and both read it before either allocates
    sp = SelfPlay(eng, games, ARGS, evaluator=ev, dirichlet_noise=True, seed=0x5EED, board_base=rank * games,
                  mem_budget=4 << 30)
    sp.reset()
    sp.run(ITERS, use_graph=True)
    ex = sp.drain()
    assert sp.capacity_events() == {"prunes": 0, "resets": 0, "unexpanded": 0}
    if dist_on:
        ex = gather_examples(ex)
    torch.cuda.synchronize(dev)
    return {k: v.cpu().numpy() for k, v in ex.items()}


def _worker(rank, world, port, out):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "alphazero-general-ori_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = _play(rank, B, net_seed=rank, dist_on=True)          # rank 1's own net is replaced
    if rank == 0:
        np.savez(out, **ex)
    dist.barrier()
    dist.destroy_process_group()


def _sorted(ex):
    m = ex["meta"]
    order = np.lexsort((m[:, 2], m[:, 1], m[:, 0]))
    return {k: v[order] for k, v in ex.items()}


def test_two_rank_selfplay_equals_one_process(tmp_path):
    world = 2
    out = str(tmp_path / "gathered.npz")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    with np.load(out) as z:
        got = {k: z[k] for k in z.files}
    ref = _play(0, world * B, net_seed=0, dist_on=False)
    assert len(ref["meta"]) > 4 * B                           # games finished on both shards
    assert (ref["meta"][:, 0] < B).any() and (ref["meta"][:, 0] >= B).any()
    assert set(got) == set(ref)
    assert len(got["meta"]) == len(ref["meta"])
    # rank order is kept: rank 0's board ids first
    ids = got["meta"][:, 0]
    assert (ids[: (ids < B).sum()] < B).all()
    g, r = _sorted(got), _sorted(ref)
    for k in ref:
        np.testing.assert_array_equal(g[k], r[k], err_msg=k)
