"""The training step's skip decisions taken on the device (adam.hip
``MauvStepGate``): a non-finite loss skips the batch (multimodal.py:133-135), non-finite
gradients skip the optimizer step AND the zero_grad (multimodal.py:141-145, so the arena keeps
them), otherwise Adam steps and the gradients are zeroed.  The gated path (FusedAdam) is held
against the host-decided path (``.item()`` decisions; FusedAdam, and the reference's own
torch.optim.Adam) over a sequence with an injected NaN input and an injected NaN gradient,
single-rank and with two gloo ranks on one GPU; the steady-state gated step is checked to make
no synchronising call (torch.cuda sync-debug mode)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

# batch kinds: "ok", "nan_loss" (one input pixel NaN), "nan_grad" (a NaN written into the
# gradient arena after the backward, before the scan)
SEQ = ["ok", "ok", "nan_loss", "ok", "nan_grad", "ok"]


def _model(seed=0):
    from mauv.models import define_models, DEFAULT_PRIOR
    torch.manual_seed(seed)
    m = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].cuda()
    return m


def _batch(seed, kind, B=2, S=64):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 3, S, S, generator=g)
    b = torch.rand(B, 3, S, S, generator=g)
    s = torch.rand(B, 1, S, S, generator=g)
    y = torch.randint(0, 7, (B,), generator=g)
    if kind == "nan_loss":
        x[0, 0, 3, 3] = float("nan")
    return x.cuda(), b.cuda(), s.cuda(), y.cuda()


def _nan_into_head_grad(model):
    """A NaN in the fusion head's last gradient (the arena slice DistributedMC reduces in
    allreduce_grads, after the backward)."""
    from mauv.engine import root_state
    from mauv.kl import unwrap
    ar = root_state(unwrap(model)).arena
    ar.flat.narrow(0, ar.offsets[-1], 1).fill_(float("nan"))   # a kernel, no host copy


class _InjectNaNGrad:
    """Write a NaN into the arena between the backward and the non-finite scan, in both the
    gated (``_count_nonfinite``) and the host-decided (``_grads_finite``) path — or, for a
    DistributedMC model, before its all-reduce (so it reaches every rank, as a real one would)."""

    def __init__(self, ddp=None):
        import mauv.train as T
        self.T, self.on, self.ddp = T, False, ddp
        self.orig_count, self.orig_finite = T._count_nonfinite, T._grads_finite
        if ddp is not None:
            orig = ddp.allreduce_grads

            def allreduce():
                if self.on:
                    _nan_into_head_grad(ddp)
                return orig()
            ddp.allreduce_grads = allreduce
            return

        def count(model, counter):
            if self.on:
                _nan_into_head_grad(model)
            return self.orig_count(model, counter)

        def finite(model):
            if self.on:
                _nan_into_head_grad(model)
            return self.orig_finite(model)
        T._count_nonfinite, T._grads_finite = count, finite

    def close(self):
        self.T._count_nonfinite, self.T._grads_finite = self.orig_count, self.orig_finite


def _run(model, opt, seq, seed0, inject, sync_check_from=None):
    from mauv.engine import root_state
    from mauv.kl import unwrap
    from mauv.train import mc_train_step
    crit = torch.nn.CrossEntropyLoss()
    st = root_state(unwrap(model))
    flags = []
    for i, kind in enumerate(seq):
        x, b, s, y = _batch(seed0 + i, kind)
        st.offset = 1000 * i          # same MC samples in both arms
        inject.on = kind == "nan_grad"
        if sync_check_from is not None and i >= sync_check_from:
            torch.cuda.synchronize()
            torch.cuda.set_sync_debug_mode("error")
        try:
            r = mc_train_step(model, (x, b, s), y, crit, opt, 2, 2, 1e-3)
        finally:
            torch.cuda.set_sync_debug_mode(0)
        inject.on = False
        if r is None:
            flags.append((False, False))
        else:
            flags.append((bool(r.get("ok_loss", True)), bool(r["stepped"])))
    torch.cuda.synchronize()
    return flags


def test_gated_step_matches_host_decided_reference(monkeypatch):
    """Three arms on the same weights, batches and MC samples: the gated step (FusedAdam), the
    host-decided step with the same FusedAdam (``.item()`` decisions, mc_train_step's other
    path) and the host-decided step with the reference's own torch.optim.Adam.  All take the
    same decisions; the two FusedAdam arms end with bit-identical parameters (the gate changes
    where the decision is taken, not the arithmetic).  torch's Adam differs in rounding, which
    Adam's first steps amplify on elements with |g| ~ eps, so that arm is held to decisions."""
    import mauv.train as T
    from mauv.optim import FusedAdam, G_POISONED, G_STEP, G_SKIP_LOSS, G_SKIP_GRAD
    from mauv.engine import root_state
    inject = _InjectNaNGrad()
    try:
        gat, host, ref = _model(), _model(), _model()
        for mm in (host, ref):
            root_state(mm).seed = root_state(gat).seed
        opt_gat = FusedAdam(gat.parameters(), lr=1e-3, weight_decay=1e-5)
        opt_host = FusedAdam(host.parameters(), lr=1e-3, weight_decay=1e-5)
        opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
        # steady-state gated steps (from the second one on) make no synchronising call
        f_gat = _run(gat, opt_gat, SEQ, 10, inject, sync_check_from=1)
        real_gate = T._step_gate
        monkeypatch.setattr(T, "_step_gate", lambda *a: None)   # the host-decided path
        f_host = _run(host, opt_host, SEQ, 10, inject)
        monkeypatch.setattr(T, "_step_gate", real_gate)
        f_ref = _run(ref, opt_ref, SEQ, 10, inject)
    finally:
        inject.close()
    want = [(True, True), (True, True), (False, False), (True, True), (True, False),
            (True, False)]   # after the NaN gradient the arena stays poisoned (no zero_grad)
    assert f_gat == want, f_gat
    assert [st for _, st in f_host] == [st for _, st in want], f_host
    assert [st for _, st in f_ref] == [st for _, st in want], f_ref
    bad = [n for (n, p), q in zip(host.named_parameters(), gat.parameters())
           if not torch.equal(p.detach(), q.detach())]
    assert not bad, bad[:5]
    # the reference keeps the skipped step's non-finite gradients; so does the arena
    assert not torch.isfinite(root_state(gat).arena.flat).all()
    assert not all(torch.isfinite(p.grad).all() for p in ref.parameters())
    gate = opt_gat._gate.cpu()
    assert int(gate[G_STEP]) == 3 and int(gate[G_POISONED]) == 1
    assert int(gate[G_SKIP_LOSS]) == 1 and int(gate[G_SKIP_GRAD]) == 2
    # the optimizer's state_dict carries the device step count, torch.optim.Adam-compatible
    sd = opt_gat.state_dict()
    assert {float(v["step"]) for v in sd["state"].values()} == {3.0}
    assert {float(v["step"]) for v in opt_host.state_dict()["state"].values()} == {3.0}
    opt_ref.load_state_dict(sd)


def test_nan_loss_batch_leaves_clean_arena_and_counts():
    """A non-finite loss on a clean arena: the batch's gradients are taken back out (the
    reference never ran that backward) and the drop-in loop does not count or log the batch."""
    from mauv.optim import FusedAdam
    from mauv.engine import root_state
    from mauv.train import train_multimodal_model
    from tests.helpers import ListLoader, NullWriter
    m = _model(1)
    opt = FusedAdam(m.parameters(), lr=1e-4)
    batches = []
    for i, kind in enumerate(["ok", "nan_loss", "ok"]):
        x, b, s, y = _batch(40 + i, kind)
        batches.append({"main_image": x.cpu(), "bathy_image": b.cpu(), "sss_image": s.cpu(),
                        "label": y.cpu(), "patch_bathy": {}, "patch_sss": {}})
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        loss, acc = train_multimodal_model(m, ListLoader(batches, 2), torch.nn.CrossEntropyLoss(),
                                           opt, 1, "cuda", "multimodal", 2, 2, NullWriter(),
                                           csv_path=os.path.join(d, "t.csv"))
    assert loss > 0 and 0.0 <= acc <= 1.0
    assert torch.isfinite(root_state(m).arena.flat).all()
    assert (root_state(m).arena.flat == 0).all()          # zeroed after the last step
    assert int(opt._gate[4].item()) == 2                   # two steps taken


def test_gate_starts_from_the_arena_state():
    """the gate takes a skipped batch's gradients back out by zeroing a CLEAN arena.
    (a) finite gradients left by a backward outside the loop: the steps take the host-decided
    path (a NaN-loss batch runs no backward and the leftovers stay, multimodal.py:133-135; the
    next good batch steps on their sum) until a zero_grad leaves the arena clean, then the gated
    path resumes; (b) an arena poisoned by an ungated skip: the gate starts poisoned, so a NaN-loss
    batch keeps the non-finite gradients instead of zeroing them."""
    import mauv.train as T
    from mauv.optim import FusedAdam, G_POISONED
    from mauv.engine import root_state
    crit = torch.nn.CrossEntropyLoss()
    m = _model(2)
    opt = FusedAdam(m.parameters(), lr=1e-4)
    x, b, s, y = _batch(60, "ok")
    T.mc_loss(m, (x, b, s), y, crit, 2, 2, 1e-3)[0].backward()   # outside the loop
    flat = root_state(m).arena.flat
    left = flat.clone()
    assert (left != 0).any()
    r = T.mc_train_step(m, _batch(61, "nan_loss")[:3], y, crit, opt, 2, 2, 1e-3)
    assert r is None and torch.equal(flat, left)            # skipped, leftovers kept
    r = T.mc_train_step(m, _batch(62, "ok")[:3], y, crit, opt, 2, 2, 1e-3)
    assert "ok_loss" not in r and r["stepped"]               # host path, stepped, zero_grad
    assert all(p.grad is None or not p.grad.any() for p in m.parameters())
    r = T.mc_train_step(m, _batch(63, "ok")[:3], y, crit, opt, 2, 2, 1e-3)
    assert "ok_loss" in r                                    # clean arena: gated again
    # (b) poisoned by an ungated skip
    m2 = _model(3)
    opt2 = FusedAdam(m2.parameters(), lr=1e-4)
    inject = _InjectNaNGrad()
    real_gate = T._step_gate
    try:
        T._step_gate = lambda *a: None
        inject.on = True
        r = T.mc_train_step(m2, _batch(64, "ok")[:3], y, crit, opt2, 2, 2, 1e-3)
        inject.on = False
        assert r is not None and not r["stepped"]
    finally:
        T._step_gate = real_gate
        inject.close()
    assert not torch.isfinite(root_state(m2).arena.flat).all()
    r = T.mc_train_step(m2, _batch(65, "nan_loss")[:3], y, crit, opt2, 2, 2, 1e-3)
    assert "ok_loss" in r and not bool(r["ok_loss"])
    assert int(opt2._gate[G_POISONED].item()) == 1
    assert not torch.isfinite(root_state(m2).arena.flat).all()   # kept, not zeroed


def test_gated_step_runs_optimizer_hooks_and_marks_the_step():
    """the gated step records torch's step flag (no scheduler warning) and runs the
    optimizer's step hooks like Optimizer.step."""
    import warnings
    from mauv.optim import FusedAdam
    from mauv.train import mc_train_step
    m = _model(4)
    opt = FusedAdam(m.parameters(), lr=1e-4)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    calls = []
    opt.register_step_pre_hook(lambda o, a, k: calls.append("pre"))
    opt.register_step_post_hook(lambda o, a, k: calls.append("post"))
    x, b, s, y = _batch(70, "ok")
    r = mc_train_step(m, (x, b, s), y, torch.nn.CrossEntropyLoss(), opt, 2, 2, 1e-3)
    assert "ok_loss" in r and calls == ["pre", "post"]
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        sched.step()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-auv_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mauv.ddp import DistributedMC
    from mauv.optim import FusedAdam
    from mauv.engine import root_state
    model = _model()
    ddp = DistributedMC(model)
    opt = FusedAdam(model.parameters(), lr=1e-3)
    inject = _InjectNaNGrad(ddp)
    # rank 0 alone sees the NaN loss (batch 2) and the NaN gradient (batch 4): every rank
    # must skip both, and the ranks stay identical
    seq = SEQ if rank == 0 else ["ok"] * len(SEQ)
    try:
        flags = _run(ddp, opt, seq, 10 + 100 * rank, inject)
    finally:
        inject.close()
    flat = torch.cat([p.detach().flatten() for p in model.parameters()]).cpu()
    torch.save((flags, flat, int(opt._gate[4].item())), os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_gated_step_two_ranks_agree():
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt")) for r in range(2)]
    want = [(True, True), (True, True), (False, False), (True, True), (True, False),
            (True, False)]
    for flags, _, step in res:
        assert flags == want, flags
        assert step == 3
    assert torch.equal(res[0][1], res[1][1])
