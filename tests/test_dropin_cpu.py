"""The drop-in loops with a foreign host model, as the reference's own unittests drive them
(unittests/test_train.py:30-78: dummy CPU modules, ``get_kl_loss`` patched to a constant at
``Multimodal_AUV.train.multimodal.get_kl_loss``).  Such models take the reference's
sequential loop and its torch maths: no host pointer may reach a HIP kernel (the process has
no GPU here, so any kernel launch would fail the test)."""
import csv
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from tests.helpers import ListLoader, NullWriter


class TinyTriModal(nn.Module):
    def __init__(self, C=3):
        super().__init__()
        self.a = nn.Linear(3 * 8 * 8, 4)
        self.b = nn.Linear(3 * 8 * 8, 4)
        self.c = nn.Linear(1 * 8 * 8, 4)
        self.out = nn.Linear(12, C)

    def forward(self, x, bathy, sss):
        f = torch.cat([self.a(x.flatten(1)), self.b(bathy.flatten(1)), self.c(sss.flatten(1))], 1)
        return self.out(f)


def _batches(n=2, B=4, C=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [{"main_image": torch.randn(B, 3, 8, 8, generator=g),
             "bathy_image": torch.rand(B, 3, 8, 8, generator=g),
             "sss_image": torch.rand(B, 1, 8, 8, generator=g),
             "label": torch.randint(0, C, (B,), generator=g),
             "patch_bathy": {}, "patch_sss": {}} for _ in range(n)]


KL = 0.05


@pytest.fixture
def patched_kl(monkeypatch):
    import Multimodal_AUV.train.multimodal as mm
    import Multimodal_AUV.train.unimodal as um
    monkeypatch.setattr(mm, "get_kl_loss", lambda model: torch.tensor(KL))
    monkeypatch.setattr(um, "get_kl_loss", lambda model: torch.tensor(KL))
    return mm, um


def test_train_multimodal_host_model(tmp_path, patched_kl):
    mm, _ = patched_kl
    torch.manual_seed(0)
    model = TinyTriModal()
    ref = TinyTriModal()
    ref.load_state_dict(model.state_dict())
    batches = _batches()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    csv_path = tmp_path / "run" / "train.csv"
    csv_path.parent.mkdir()
    loss, acc = mm.train_multimodal_model(model, ListLoader(batches, 4), nn.CrossEntropyLoss(),
                                          opt, epoch=1, device=torch.device("cpu"),
                                          model_type="multimodal", total_num_epochs=3, num_mc=3,
                                          sum_writer=NullWriter(), csv_path=str(csv_path))
    # the reference's maths (multimodal.py:107-146) on the twin model: the dummy model is
    # deterministic, so the MC mean is the single output
    kw = 2 ** 2 / 2 ** 3
    tot, correct = 0.0, 0
    for b in batches:
        out = torch.stack([ref(b["main_image"], b["bathy_image"], b["sss_image"])
                           for _ in range(3)]).mean(0)
        lo = F.cross_entropy(out, b["label"]) + KL / 4 * kw
        lo.backward()
        ropt.step()
        ropt.zero_grad()
        tot += lo.item()
        correct += int((out.argmax(1) == b["label"]).sum())
    assert loss == pytest.approx(tot / 8, rel=1e-6)
    assert acc == correct / 8
    for p, q in zip(model.parameters(), ref.parameters()):
        assert torch.allclose(p, q, atol=1e-7)
    rows = list(csv.reader(open(csv_path)))
    assert rows[1][:2] == ["1", "multimodal"] and float(rows[1][5]) == pytest.approx(KL / 4 * kw)


def test_nan_loss_skips_batch_on_host(tmp_path, patched_kl, monkeypatch):
    mm, _ = patched_kl
    monkeypatch.setattr(mm, "get_kl_loss", lambda model: torch.tensor(float("nan")))
    model = TinyTriModal()
    before = [p.detach().clone() for p in model.parameters()]
    csv_path = tmp_path / "run" / "train.csv"
    csv_path.parent.mkdir()
    loss, acc = mm.train_multimodal_model(model, ListLoader(_batches(), 4), nn.CrossEntropyLoss(),
                                          torch.optim.Adam(model.parameters()), epoch=0,
                                          device=torch.device("cpu"), model_type="m",
                                          total_num_epochs=2, num_mc=2, sum_writer=NullWriter(),
                                          csv_path=str(csv_path))
    # every batch skipped -> the reference divides by zero and its except returns zeros
    assert (loss, acc) == (0.0, 0.0)
    for p, q in zip(model.parameters(), before):
        assert torch.equal(p, q)


def test_evaluate_multimodal_host_model(tmp_path, patched_kl):
    mm, _ = patched_kl
    torch.manual_seed(1)
    model = TinyTriModal()
    batches = _batches(seed=3)
    csv_path = tmp_path / "run" / "test.csv"
    csv_path.parent.mkdir()
    acc = mm.evaluate_multimodal_model(model, ListLoader(batches, 4), torch.device("cpu"),
                                       epoch=0, total_num_epochs=2, num_mc=2,
                                       model_type="multimodal", csv_path=str(csv_path))
    with torch.no_grad():
        outs = [model(b["main_image"], b["bathy_image"], b["sss_image"]) for b in batches]
    correct = sum(int((o.argmax(1) == b["label"]).sum()) for o, b in zip(outs, batches))
    assert acc == correct / 8
    row = list(csv.reader(open(csv_path)))[1]
    P = torch.cat([F.softmax(o, 1) for o in outs])
    H = -(P * torch.log(P + 1e-8)).sum(1)
    assert float(row[4]) == pytest.approx(H.mean().item(), rel=1e-5)
    assert abs(float(row[5])) < 1e-6     # deterministic model: no epistemic part


def test_predict_host_model(tmp_path):
    import Multimodal_AUV.inference.predictors as pr
    torch.manual_seed(2)
    model = TinyTriModal()
    b = _batches(1, seed=5)[0]
    loader = [(b["main_image"], b["bathy_image"], b["sss_image"], [f"n{i}" for i in range(4)])]
    path = tmp_path / "pred.csv"
    pr.multimodal_predict_and_save(model, loader, torch.device("cpu"), str(path),
                                   num_mc_samples=3)
    rows = list(csv.reader(open(path)))
    assert rows[0] == ["Image Name", "Predicted Class", "Predictive Uncertainty",
                       "Aleatoric Uncertainty"]
    assert [r[0] for r in rows[1:]] == ["n0", "n1", "n2", "n3"]
    with torch.no_grad(), torch.amp.autocast(device_type="cpu"):
        P = F.softmax(model(b["main_image"], b["bathy_image"], b["sss_image"]), 1).float()
    for i, r in enumerate(rows[1:]):
        assert int(r[1]) == int(P[i].argmax())
        assert float(r[2]) == 0.0
        h = -(P[i] * torch.log(P[i] + 1e-7)).sum().item()
        assert abs(float(r[3]) - h) < 1e-2 and math.isfinite(float(r[3]))


def test_unimodal_host_model(tmp_path, patched_kl):
    _, um = patched_kl

    class Uni(nn.Module):
        def __init__(self):
            super().__init__()
            self.f = nn.Linear(3 * 8 * 8, 3)

        def forward(self, x):
            return self.f(x.flatten(1))
    model = Uni()
    csv_path = tmp_path / "run" / "uni.csv"
    csv_path.parent.mkdir()
    acc, loss = um.train_unimodal_model(model, ListLoader(_batches(), 4), nn.CrossEntropyLoss(),
                                        torch.optim.Adam(model.parameters()), epoch=0,
                                        total_num_epochs=2, num_mc=2, sum_writer=NullWriter(),
                                        device=torch.device("cpu"), model_type="image",
                                        csv_path=str(csv_path))
    assert loss > 0 and 0.0 <= acc <= 1.0
    acc2 = um.evaluate_unimodal_model(model, ListLoader(_batches(seed=9), 4),
                                      torch.device("cpu"), epoch=0, csv_path=str(csv_path),
                                      total_num_epochs=2, num_mc=2, model_type="image")
    assert 0.0 <= acc2 <= 1.0
    row = list(csv.reader(open(csv_path)))[-1]
    assert float(row[4]) == 0.0   # deterministic model: zero MC variance


def test_mauv_model_on_host_refuses_kernels():
    """A mauv Bayesian model left on the host fails loudly instead of launching kernels on
    host pointers."""
    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.kl import get_kl_loss
    m = define_models(None, 7, DEFAULT_PRIOR)["image_model"]
    with pytest.raises(RuntimeError, match="ROCm"):
        get_kl_loss(m)
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.zeros(2, 3, 32, 32))
    from mauv import ops
    with pytest.raises(ValueError):
        ops.nonfinite_count(torch.zeros(4), torch.zeros(1, dtype=torch.int32))
