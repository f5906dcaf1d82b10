"""Multi-rank paths on CPU with the gloo backend (world size 2): board sharding by global
id is invariant to the number of ranks, the episode-end example all-gather
(splendor.selfplay.gather_examples) concatenates every rank's examples in rank order, and
the network broadcast (splendor.selfplay.broadcast_network) leaves every rank with rank
0's weights."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, T, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "alphazero-general-ori_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import _oracle as O
    from splendor.selfplay import gather_examples
    # 1) env shard: boards [rank*B, (rank+1)*B), keyed by global id
    r = O.rollout_run(2, B, T, 0x5EED, board_base=rank * B)
    st = torch.from_numpy(r["state"])
    parts = [torch.zeros_like(st) for _ in range(world)]
    dist.all_gather(parts, st)
    # 2) example exchange: rank-dependent counts
    k = 3 + 2 * rank
    ex = {"board": torch.full((k, 56, 7), rank, dtype=torch.int8),
          "pi": torch.arange(k * 409, dtype=torch.float32).reshape(k, 409) + 1000 * rank,
          "winner": torch.full((k, 2), float(rank))}
    got = gather_examples(ex)
    # 3) network broadcast: differently seeded nets end up equal to rank 0's
    from splendor.nnet import SplendorNNet
    from splendor.selfplay import broadcast_network
    torch.manual_seed(100 + rank)
    net = SplendorNNet(2)
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.fill_(0.1 * (rank + 1))
    broadcast_network(net)
    flat = torch.cat([t.reshape(-1).float() for t in net.state_dict().values()])
    nets = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(nets, flat)
    torch.manual_seed(100)
    ref = SplendorNNet(2)
    for m in ref.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.fill_(0.1)
    ref_flat = torch.cat([t.reshape(-1).float() for t in ref.state_dict().values()])
    if rank == 0:
        q.put((torch.cat(parts).numpy(), {kk: v.numpy() for kk, v in got.items()},
               [x.numpy() for x in nets], ref_flat.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_example_allgather():
    B, T, world = 64, 48, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    states, ex, nets, ref_net = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    single = O.rollout_run(2, world * B, T, 0x5EED)
    np.testing.assert_array_equal(states, single["state"])
    assert ex["board"].shape[0] == 3 + 5
    assert (ex["board"][:3] == 0).all() and (ex["board"][3:] == 1).all()
    np.testing.assert_array_equal(ex["pi"][3:], np.arange(5 * 409, dtype=np.float32).reshape(5, 409) + 1000)
    np.testing.assert_array_equal(nets[0], ref_net)
    np.testing.assert_array_equal(nets[1], ref_net)
