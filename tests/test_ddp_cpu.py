"""world_size-2 gloo tests on CPU for the N>1 paths: the flat-arena gradient all-reduce of
mauv.ddp.DistributedMC (training) and the MC-sharded sufficient-statistics all-reduce
(inference).  The HIP compute itself is exercised by the -m gpu tests."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _ddp_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "multimodal-auv_amd")]
    _init(rank, world, port)
    from mauv.ddp import DistributedMC
    from mauv.engine import root_state
    torch.manual_seed(rank)  # different init per rank: the wrapper must broadcast rank 0's
    net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 3))
    ddp = DistributedMC(net, bucket_bytes=16)  # tiny buckets: exercise the bucket loop
    st = root_state(net)
    arena = st.grads(torch.device("cpu"))
    for i, p in enumerate(net.parameters()):
        p.grad.fill_(float(rank + 1) * (i + 1))
    ddp.allreduce_grads()
    torch.save((rank, [p.detach().clone() for p in net.parameters()],
                [p.grad.clone() for p in net.parameters()], st.seed, arena.flat.numel()),
               os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def _run(worker, tmp_path, world=2):
    mp.spawn(worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    return [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=False)
            for r in range(world)]


def test_distributed_mc_allreduce_and_broadcast(tmp_path):
    res = _run(_ddp_worker, tmp_path)
    (_, p0, g0, s0, n0), (_, p1, g1, s1, n1) = res
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)  # parameters broadcast from rank 0
    for i, (a, b) in enumerate(zip(g0, g1)):
        assert torch.equal(a, b)
        assert torch.allclose(a, torch.full_like(a, 1.5 * (i + 1)))  # mean of (1, 2) x (i+1)
    assert s0 != s1  # per-rank Philox streams (each replica samples its own epsilons)
    assert n0 == n1 == 5 * 7 + 7 + 7 * 3 + 3


def _stats_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-auv_amd")]
    from mauv.predict import local_mc_count
    _init(rank, world, port)
    torch.manual_seed(0)
    N, B, C = 7, 3, 4
    logits = torch.randn(N, B, C, dtype=torch.float64)
    # rank r takes MC samples [start, start+local) exactly as mauv.predict shards them
    local = local_mc_count(N, rank, world)
    start = sum(local_mc_count(N, r, world) for r in range(rank))
    P = torch.softmax(logits[start:start + local], -1)
    sums = torch.cat([P.sum(0), (P * P).sum(0),
                      (-(P * torch.log(P + 1e-7)).sum(-1)).sum(0, keepdim=True).T], 1)
    dist.all_reduce(sums)
    torch.save((rank, sums), os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_mc_sharded_statistics_equal_single_process(tmp_path):
    sums = [r[1] for r in _run(_stats_worker, tmp_path)]
    assert torch.equal(sums[0], sums[1])
    torch.manual_seed(0)
    N, B, C = 7, 3, 4
    P = torch.softmax(torch.randn(N, B, C, dtype=torch.float64), -1)
    s = sums[0]
    mean = s[:, :C] / N
    var = ((s[:, C:2 * C] - N * mean * mean) / (N - 1)).mean(1)
    np.testing.assert_allclose(mean.numpy(), P.mean(0).numpy(), atol=1e-12)
    np.testing.assert_allclose(var.numpy(), torch.var(P, 0).mean(1).numpy(), atol=1e-12)
    alea = s[:, 2 * C] / N
    np.testing.assert_allclose(alea.numpy(),
                               torch.mean(-torch.sum(P * torch.log(P + 1e-7), -1), 0).numpy(),
                               atol=1e-12)
