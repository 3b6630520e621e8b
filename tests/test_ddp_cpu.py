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
    assert n0 == n1 == 36 + 8 + 24 + 4   # 5*7, 7, 7*3, 3 floats, each view padded to 4


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


def _arena_worker(rank, world, port, q):
    """The tri-modal model's real arena (696 tensors, 146.8 M floats) on CPU: the trunk
    slices all-reduce from the engine's per-trunk hook (the first one before the KL backward
    has been issued, so it is deferred), the rest in allreduce_grads."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-auv_amd")]
    _init(rank, world, port)
    torch.set_num_threads(2)
    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.ddp import DistributedMC
    from mauv.engine import root_state
    torch.manual_seed(rank)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"]
    ddp = DistributedMC(model)
    st = root_state(model)
    arena = st.grads(torch.device("cpu"))
    assert len(arena.params) == 696 and all(o % 4 == 0 for o in arena.offsets)
    for i, p in enumerate(model.parameters()):
        p.grad.fill_(float(rank + 1) * (i % 7 + 1))
    with torch.enable_grad():
        ddp._begin_step()
    trunks = (model.image_model_feat, model.bathy_model_feat, model.sss_model_feat)
    st.grad_ready_hook(trunks[0])          # before the KL backward: deferred
    st.kl_bwd_count += 1                   # (what mauv.kl's backward does)
    st.grad_ready_hook(trunks[1])
    st.grad_ready_hook(trunks[2])
    early = sorted(ddp._done)
    ddp.allreduce_grads()
    ok = all(torch.all(p.grad == 1.5 * (i % 7 + 1)).item()
             for i, p in enumerate(model.parameters()))
    head = sum(p.numel() for n, p in model.named_parameters()
               if not n.split(".")[0].endswith("_feat"))
    p0 = model.fc2.mu_weight.detach().clone()
    torch.save((ok, early, arena.numel, head, p0), os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_trimodal_arena_per_trunk_allreduce(tmp_path):
    res = _run(_arena_worker, tmp_path)
    for ok, early, numel, head, _ in res:
        assert ok
        assert len(early) == 2          # bathy and sss slices overlapped; image deferred
        for a, b in early:
            assert b - a >= 23_000_000 * 2   # one trunk's mu + rho
        assert early[0][1] <= early[1][0]
    assert torch.equal(res[0][4], res[1][4])   # rank 0's parameters broadcast


def _nan_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-auv_amd")]
    _init(rank, world, port)
    from mauv.ddp import DistributedMC
    from mauv.train import mc_train_step
    torch.manual_seed(0)

    class Tri(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.f = torch.nn.Linear(12, 3)

        def forward(self, x, b, s):
            return self.f(torch.cat([x, b, s], 1))
    net = Tri()
    ddp = DistributedMC(net)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    x = torch.randn(4, 4)
    if rank == 1:
        x[0, 0] = float("nan")          # only rank 1 sees a non-finite loss
    before = [p.detach().clone() for p in net.parameters()]
    r1 = mc_train_step(ddp, (x, torch.randn(4, 4), torch.randn(4, 4)), torch.tensor([0, 1, 2, 0]),
                       torch.nn.CrossEntropyLoss(), opt, 2, 4, 0.5)
    same = all(torch.equal(a, b) for a, b in zip(before, net.parameters()))
    x2 = torch.full((4, 4), float(rank + 1))   # finite everywhere: both step, grads averaged
    r2 = mc_train_step(ddp, (x2, torch.zeros(4, 4), torch.zeros(4, 4)), torch.tensor([0, 1, 2, 0]),
                       torch.nn.CrossEntropyLoss(), opt, 2, 4, 0.5)
    params = [p.detach().clone() for p in net.parameters()]
    torch.save((r1 is None, same, r2 is not None and r2["stepped"], params),
               os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_nan_loss_on_one_rank_skips_on_all(tmp_path):
    """A non-finite loss on one rank skips the batch on every rank (no unpaired all-reduce);
    the next finite batch steps everywhere with averaged gradients (identical parameters)."""
    res = _run(_nan_worker, tmp_path)
    for skipped, same, stepped, _ in res:
        assert skipped and same and stepped
    for a, b in zip(res[0][3], res[1][3]):
        assert torch.equal(a, b)


def _bf16_worker(rank, world, port, q):
    """grad_dtype=bf16: the exchange moves bf16 (half the bytes of the fp32 arena); the
    averaged fp32 gradients equal the fp32 exchange's within bf16 rounding of each rank's
    contribution, on every rank bit-identically."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-auv_amd")]
    _init(rank, world, port)
    from mauv.ddp import DistributedMC
    from mauv.engine import root_state
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(50, 70), torch.nn.Linear(70, 30))
    ddp = DistributedMC(net, bucket_bytes=1000, grad_dtype=torch.bfloat16)
    assert ddp.bucket_elems == 500      # bf16 buckets hold twice the values of fp32 ones
    st = root_state(net)
    st.grads(torch.device("cpu"))
    g = torch.Generator().manual_seed(10 + rank)
    local = [torch.randn(p.shape, generator=g) * (rank + 1) for p in net.parameters()]
    for p, v in zip(net.parameters(), local):
        p.grad.copy_(v)
    ddp.allreduce_grads()
    torch.save(([p.grad.clone() for p in net.parameters()], local, ddp._lp.dtype),
               os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_bf16_gradient_exchange(tmp_path):
    res = _run(_bf16_worker, tmp_path)
    (g0, l0, dt0), (g1, l1, _) = res
    assert dt0 == torch.bfloat16
    for a, b, x, y in zip(g0, g1, l0, l1):
        assert torch.equal(a, b)                       # every rank holds the same average
        exact = (x + y) / 2
        # each contribution rounded to bf16 (2^-9 relative), the sum rounded once more
        tol = (x.abs() + y.abs()) * 2.0 ** -8 / 2 + exact.abs() * 2.0 ** -8
        assert ((a - exact).abs() <= tol + 1e-12).all()
        assert not torch.equal(a, exact)               # it really went through bf16
